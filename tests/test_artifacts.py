"""Consistency of the committed measurement artifacts (profiles/): the latest bench line keeps the bench.py
contract, its roofline fields are self-consistent, and the roofline kernel's average launch duration
(HIP events inside bench.py) agrees with the rocprofv3 --kernel-trace --stats summary of the same command."""
import csv
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def _latest(pattern):
    files = sorted(glob.glob(os.path.join(PROF, pattern)))
    assert files, pattern
    return files[-1]


def test_bench_line_contract():
    b = json.load(open(_latest("r*_bench.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in b, k
    assert b["higher_is_better"] is True and b["scaling"] == "weak"
    # value = frames (N*T) per second at N=64, T=300
    assert abs(b["value"] - 64 * 300 * b["n_gpus"] / (b["ms_per_step"] / 1e3)) / b["value"] < 0.01
    r = b["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["peak"] > 0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["traffic"] is None or r["traffic"] > 0
    c = b["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0 and c["sample"]


def test_roofline_kernel_matches_rocprof():
    bench = _latest("r*_bench.json")
    tag = os.path.basename(bench).split("_")[0]
    stats = os.path.join(PROF, f"{tag}_bench_kernel_stats.csv")
    assert os.path.exists(stats), stats
    b = json.load(open(bench))
    m = re.match(r"(\w+)(?:<([^>]*)>)?", b["roofline"]["kernel"])
    name = m.group(1)
    if b["roofline"].get("rocprof_kernels"):  # a kernel family: the call-weighted mean over its kernels' rows
        names = b["roofline"]["rocprof_kernels"]
        rows = [r for r in csv.DictReader(open(stats))
                if any(re.search(r"\b" + re.escape(n) + r"[<(]", r["Name"]) for n in names)]
        assert rows, names
        prof_ms = sum(float(r["TotalDurationNs"]) for r in rows) / sum(int(r["Calls"]) for r in rows) / 1e6
        assert abs(prof_ms - b["roofline"]["avg_launch_ms"]) / prof_ms < 0.10
        return
    if m.group(2) is not None:
        # the bench names the leading template arguments; the trailing (defaulted) ones may be omitted
        targs = [t.strip() for t in m.group(2).split(",")]
        want = f"{name}<{', '.join(targs)}"
        rows = [r for r in csv.DictReader(open(stats)) if re.search(re.escape(want) + r"[,>]", r["Name"])]
    else:  # every instantiation of the named kernel (the bench brackets all of its launches)
        rows = [r for r in csv.DictReader(open(stats)) if re.search(r"\b" + re.escape(name) + r"[<(]", r["Name"])]
        want = name
    assert rows, want
    prof_ms = float(rows[0]["AverageNs"]) / 1e6
    assert abs(prof_ms - b["roofline"]["avg_launch_ms"]) / prof_ms < 0.10
