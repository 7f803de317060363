#!/usr/bin/env python3
"""GPU box tool: bench.py's MultiwayMerge sample alone (for rocprofv3 --pmc passes over the merge
kernels).   python tools/merge_sample.py SCALE FRAC STEPS"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0 / 16
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    import torch

    torch.cuda.set_device(0)
    import bench
    import combblas_amd as cb

    print(json.dumps(bench.merge_measurement(cb.rmat(scale, 16, dtype=np.float64), frac, steps)), flush=True)


if __name__ == "__main__":
    main()
