"""GPU busy time vs wall time per training step from a rocprofv3 kernel trace (--kernel-trace, csv).

Steps are delimited by the optimizer (the Adam launch(es) end every step: the package's adam_kernel, or torch's multi_tensor_apply).  For the
last `n` complete steps it prints: wall time (first kernel start -> last kernel end), GPU busy time (union of
all kernel intervals, so overlapping streams count once), the sum of kernel durations, and the launch count.
busy << wall means the step waits on the host (launch-bound); sum >> busy means the streams overlap.

    python tools/trace_gaps.py gpurun_out/prof_x/<host>/<pid>_kernel_trace.csv [n]
"""
import csv
import glob
import os
import sys


def load(path):
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    return ks


def steps(ks):
    """Split the trace after the last Adam launch of each group of consecutive Adam launches."""
    out, cur, in_adam = [], [], False
    for k in ks:
        adam = "multi_tensor_apply" in k[2] or "fused_adam" in k[2].lower() or "adam_kernel" in k[2]
        if in_adam and not adam:
            out.append(cur)
            cur = []
        cur.append(k)
        in_adam = adam
    if cur and in_adam:
        out.append(cur)
    return out


def busy(ks):
    tot, end = 0, None
    for s, e, _ in sorted(ks):
        if end is None or s > end:
            tot += e - s
            end = e
        elif e > end:
            tot += e - end
            end = e
    return tot


if __name__ == "__main__":
    ks = load(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    st = steps(ks)
    # drop the first step (may start mid-warm-up) and keep the last n
    sel = st[-n:]
    for i, s in enumerate(sel):
        wall = s[-1][1] - s[0][0]
        print(f"step {i}: wall {wall / 1e6:.3f} ms  busy {busy(s) / 1e6:.3f} ms  sum {sum(e - b for b, e, _ in s) / 1e6:.3f} ms"
              f"  launches {len(s)}")
    if sel:
        w = sum(s[-1][1] - s[0][0] for s in sel) / len(sel)
        b = sum(busy(s) for s in sel) / len(sel)
        print(f"mean: wall {w / 1e6:.3f} ms, busy {b / 1e6:.3f} ms ({100 * b / w:.1f} %), launches "
              f"{sum(len(s) for s in sel) / len(sel):.0f}")
