"""Per-kernel time per step from a rocprofv3 kernel trace (steps split at the optimizer, tools/trace_gaps.py).
    python tools/kbreak.py <trace dir or csv> [steps=5] [top=40] [--diff other_trace]"""
import sys
from collections import defaultdict

import trace_gaps as T


def table(path, n):
    st = T.steps(T.load(path))[-n:]
    d = defaultdict(lambda: [0, 0])
    for s in st:
        for b, e, name in s:
            d[name][0] += e - b
            d[name][1] += 1
    return {k: (v[0] / n / 1e6, v[1] / n) for k, v in d.items()}


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[1]) if len(args) > 1 else 5
    top = int(args[2]) if len(args) > 2 else 40
    a = table(args[0], n)
    b = table(sys.argv[sys.argv.index("--diff") + 1], n) if "--diff" in sys.argv else None
    keys = sorted(a, key=lambda k: -a[k][0])[:top]
    if b:
        keys = sorted(set(a) | set(b), key=lambda k: -abs(a.get(k, (0, 0))[0] - b.get(k, (0, 0))[0]))[:top]
    for k in keys:
        ta, ca = a.get(k, (0.0, 0))
        line = "%7.3f ms %5.1f/step" % (ta, ca)
        if b:
            tb, cb = b.get(k, (0.0, 0))
            line += "  | other %7.3f ms %5.1f/step  delta %+7.3f" % (tb, cb, ta - tb)
        print(line, " ", k[:100])
    print("total %.3f ms" % sum(v[0] for v in a.values()) + (" other %.3f" % sum(v[0] for v in b.values()) if b else ""))
