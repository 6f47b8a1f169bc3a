"""FETCH_SIZE calibration for kfac_factor_tiles_x3's access pattern (buffer_load_dword,
32 lanes x 4 B = one 128-B row piece per half-wave): one 64-column factor (one tile)
over `rows` rows, every operand byte read exactly once per launch by one workgroup's
K-chunk (no re-reads), operand larger than the Infinity Cache.  Run under rocprofv3
--pmc FETCH_SIZE: FETCH_SIZE x 1024 / operand bytes is the counter's scale for this
pattern.  GPU only.

    KFAC_TILES_X3=1 python tools/fetch_calib.py [rows]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bnn_kfac_amd import _native as N  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2 * 1024 * 1024
    dev = torch.device("cuda:0")
    x = torch.rand(rows, 64, device=dev)
    F = torch.zeros(64, 64, device=dev)
    op = N.rowmajor_operand(x, has_ones=False)
    job = [N.factor_job(op, F, 1.0 / rows, 0.0)]
    for _ in range(3):
        N.factor_update(job, dev)
    torch.cuda.synchronize()
    print(f"operand bytes {x.numel() * 4}")


if __name__ == "__main__":
    main()
