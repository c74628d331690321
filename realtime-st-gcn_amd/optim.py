"""Adam as one HIP launch per step (csrc/adam.hip, stgcn_adam_step).

The reference trains with ``torch.optim.Adam(model.parameters(), lr=learning_rate)`` (processor.py:579) and
steps it every ``batch_size`` trials (processor.py:561).  ``Adam`` here is a drop-in for that optimizer: the same
constructor arguments, update rule, ``param_groups`` / ``state`` (``step``, ``exp_avg``, ``exp_avg_sq``) and
state_dict, but the moments of a parameter group live in two flat fp32 buffers and the whole group is updated
by ONE kernel launch per 256 tensors (torch's fused multi-tensor Adam takes three launches for the config-2
model plus the step-counter updates).  The step counters live on the device (one slot per 2048-element block), so a step
can be captured into a HIP graph (``parallel.GraphedStep``) without ``capturable`` bookkeeping.
No CPU fallback: parameters must be fp32 HIP tensors.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L
from . import native as K

MAXT = 256  # STGCN_ADAM_MAXT: tensors per launch (gradient pointers travel as kernel arguments)


def _offsets(fs):
    out, o = [], 0
    for f in fs:
        out.append(o)
        o += f.n
    return out


class _Flat:
    """Flat state of one parameter group: moment buffers, per-block step slots, the device entry table."""

    def __init__(self, params, state):
        dev = params[0].device
        for p in params:
            if p.device != dev or p.dtype != torch.float32 or not p.is_contiguous():
                raise RuntimeError("stgcn_amd.optim.Adam: parameters must be contiguous fp32 tensors on one HIP device")
        offs, off = [], 0
        for p in params:
            offs.append(off)
            off += -(-p.numel() // 4) * 4  # 16-B aligned slices
        self.m = torch.zeros(max(off, 4), dtype=torch.float32, device=dev)
        self.v = torch.zeros_like(self.m)
        lib = L.lib()
        blocks = [int(lib.stgcn_adam_blocks(max(p.numel(), 1))) for p in params]
        self.nblocks = sum(blocks)
        self.steps = torch.zeros(self.nblocks, dtype=torch.float32, device=dev)
        ents, b0 = (L.AdamEntry * len(params))(), 0
        self.b0 = []
        for k, p in enumerate(params):
            n, o = p.numel(), offs[k]
            m, v = self.m[o:o + n], self.v[o:o + n]
            st = state.get(p, {})
            if "exp_avg" in st:  # carried over (load_state_dict, or a rebuild after parameters moved)
                m.copy_(st["exp_avg"].reshape(-1))
                v.copy_(st["exp_avg_sq"].reshape(-1))
                self.steps[b0:b0 + blocks[k]] = float(st["step"])
            e = ents[k]
            e.p, e.m, e.v, e.n, e.b0 = p.data_ptr(), m.data_ptr(), v.data_ptr(), n, b0
            e.vec = int(p.data_ptr() % 16 == 0 and m.data_ptr() % 16 == 0 and v.data_ptr() % 16 == 0)
            state[p] = {"step": self.steps[b0], "exp_avg": m.view_as(p), "exp_avg_sq": v.view_as(p)}
            self.b0.append(b0)
            b0 += blocks[k]
        self.table = torch.frombuffer(bytearray(bytes(memoryview(ents).cast("B"))), dtype=torch.uint8).to(dev)
        self.key = tuple(p.data_ptr() for p in params)
        self.n = len(params)
        self.grads = (ctypes.c_void_p * self.n)()


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False) with the update of each parameter group in one HIP launch."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("stgcn_amd.optim.Adam: amsgrad is not implemented (the reference does not use it)")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False))
        self._flat = {}

    def _flat_of(self, gi, group):
        """The flat states of a group: one per chunk of <= STGCN_ADAM_MAXT tensors (one launch each)."""
        params = group["params"]
        fs = self._flat.get(gi)
        if fs is None or sum(f.n for f in fs) != len(params) or \
                any(f.key != tuple(p.data_ptr() for p in params[o:o + f.n]) for f, o in zip(fs, _offsets(fs))):
            dev = params[0].device
            if any(p.device != dev for p in params):
                # every chunk of a group launches on one device's stream (step())
                raise RuntimeError("stgcn_amd.optim.Adam: all parameters of a group must be on one HIP device")
            fs = [_Flat(params[o:o + MAXT], self.state) for o in range(0, len(params), MAXT)]
            self._flat[gi] = fs
        return fs

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        # copy the loaded exp_avg / exp_avg_sq / step into flat buffers NOW: torch hands over the source
        # optimizer's own tensors when device and dtype already match, and they may change before our next step
        self._flat = {}
        for gi, group in enumerate(self.param_groups):
            if group["params"]:
                self._flat_of(gi, group)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = group["params"]
            if not params:
                continue
            keep, updated = [], []
            b1, b2 = group["betas"]
            for f, o in zip(self._flat_of(gi, group), _offsets(self._flat[gi])):
                for k, p in enumerate(params[o:o + f.n]):
                    g = p.grad
                    if g is None:
                        f.grads[k] = None
                        continue
                    updated.append(p)
                    if g.is_sparse or g.dtype != torch.float32 or g.shape != p.shape:
                        raise RuntimeError("stgcn_amd.optim.Adam: dense fp32 gradients of the parameter's shape only")
                    if not g.is_contiguous():
                        g = g.contiguous()
                        keep.append(g)
                    f.grads[k] = g.data_ptr()
                with K.device_of(params[0]):
                    L.check(L.lib().stgcn_adam_step(f.table.data_ptr(), f.n, f.nblocks, f.grads, f.steps.data_ptr(),
                                                    float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                                    float(group["weight_decay"]), L.stream()), "adam_step")
            # the kernel writes the parameters through raw pointers: bump their in-place version counters as
            # an aten in-place update would, so caches keyed on (storage, _version) — the fused-inference and
            # RT packs — see the new weights
            torch._C._increment_version(updated)
        return loss
