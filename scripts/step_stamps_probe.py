"""Where an LML sweep step's time goes (MPO_FIT_DEBUG=24, diagnostics only):
sw_step_kernel's step 2 of theta 0 stamps the workgroups' entry / exit (wall
clock, 100 MHz) and workgroup 0's shader cycles to the end of the pivot sweep
and from there to its exit; step 1's last exit gives the launch gap.

    MPO_FIT_DEBUG=24 python scripts/step_stamps_probe.py [n ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd import gp_fit as GF  # noqa: E402


def acc_offset(n, d):
    al = lambda x: (x + 31) & ~31   # noqa: E731
    np_ = (n + 31) // 32 * 32
    return al(n * d) + al(np_) + np_ * np_ + 2 * np_ * 32 + 32 * 32


def main():
    assert os.environ.get("MPO_FIT_DEBUG") == "24", "run with MPO_FIT_DEBUG=24"
    ns = [int(v) for v in sys.argv[1:]] or [288, 448]
    d = 5
    for n in ns:
        rng = np.random.RandomState(0)
        X = rng.rand(n, d)
        yn, _, _ = GF.normalize_targets(np.sin(X @ rng.randn(d)))
        lml = GF.DeviceLML(X, yn, device="cuda:0")
        th = np.zeros((3, d + 2))
        lml.evaluate(th)      # allocates the workspace
        base = (lml.ws.data_ptr() + 255) // 256 * 256 - lml.ws.data_ptr()
        off = base + 8 * (acc_offset(n, d) + 8)
        rows = []
        for r in range(60):
            lml.evaluate(th)
            torch.cuda.synchronize()
            st = lml.ws[off:off + 7 * 8].view(torch.int64).cpu().numpy()
            if r >= 10:
                rows.append(st)
        a = np.array(rows, dtype=np.float64)
        ten_ns = 10.0 / 1e3   # 100 MHz ticks -> us
        print(f"n={n}: step 2 of {(n + 31) // 32}: launch gap (step 1 last exit -> first entry) "
              f"{np.median(a[:, 0] - a[:, 6]) * ten_ns:.2f} us, entry spread {np.median(a[:, 1] - a[:, 0]) * ten_ns:.2f} us, "
              f"first entry -> last exit {np.median(a[:, 3] - a[:, 0]) * ten_ns:.2f} us, "
              f"exit spread {np.median(a[:, 3] - a[:, 2]) * ten_ns:.2f} us; workgroup 0: sweep {np.median(a[:, 4]):.0f} cycles, "
              f"rest {np.median(a[:, 5]):.0f} cycles", flush=True)


if __name__ == "__main__":
    main()
