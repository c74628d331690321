"""The multi-GPU bench path (`bench.py --gpus N`, what the driver's scaling run launches) rehearsed on the test box's
one GPU: STGCN_BENCH_REHEARSE=1 puts both ranks on GPU 0 over gloo.  `bench.py --gpus 2` must spawn its ranks, run
DDP, meet at the barriers and have rank 0 print exactly one JSON line with the whole-job fields (the numbers of two
ranks timesharing one GPU are not a measurement)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("extra", [[], ["--config", "4"], ["--sync-bn"]])
def test_bench_two_ranks_rehearsal(extra):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, STGCN_BENCH_REHEARSE="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-layer-roofline", "--kernel-steps", "0"] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["parallelism"].startswith("dp2") and "REHEARSAL" in d["config"]["parallelism"]
    assert d["config"]["bn_stats"] == ("sync (all ranks)" if "--sync-bn" in extra else "per-replica")
