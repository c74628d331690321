"""The north_star layer's forward alone (bench.layer_roofline): LayerNorm one-kernel vs unfused (BatchNorm: unfused only), for rocprofv3."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    pkg = ge.load_package()
    dev = torch.device("cuda", 0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    norm = sys.argv[2] if len(sys.argv) > 2 else "LayerNorm"
    print(json.dumps(bench.layer_roofline(pkg, dev, reps=reps, norm=norm)))
