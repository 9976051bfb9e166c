"""Where sw_pairs_final_kernel's time goes (MPO_FIT_DEBUG=25, diagnostics only):
theta 0's workgroups stamp their entry (first / last, wall clock 100 MHz), the
moment the last of them has its partial row written, the last workgroup's start
of the fixed-order sum (after the arrival counter) and its end.

    MPO_FIT_DEBUG=25 python scripts/pair_stamps_probe.py [n ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd import gp_fit as GF  # noqa: E402
from scripts.step_stamps_probe import acc_offset  # noqa: E402


def main():
    assert os.environ.get("MPO_FIT_DEBUG") == "25", "run with MPO_FIT_DEBUG=25"
    ns = [int(v) for v in sys.argv[1:]] or [288, 448]
    d = 5
    for n in ns:
        rng = np.random.RandomState(0)
        X = rng.rand(n, d)
        yn, _, _ = GF.normalize_targets(np.sin(X @ rng.randn(d)))
        lml = GF.DeviceLML(X, yn, device="cuda:0")
        th = np.zeros((3, d + 2))
        lml.evaluate(th)
        base = (lml.ws.data_ptr() + 255) // 256 * 256 - lml.ws.data_ptr()
        off = base + 8 * (acc_offset(n, d) + 20)
        rows = []
        for r in range(60):
            lml.evaluate(th)
            torch.cuda.synchronize()
            st = lml.ws[off:off + 5 * 8].view(torch.int64).cpu().numpy()
            if r >= 10:
                rows.append(st)
        a = np.array(rows, dtype=np.float64) * 0.01   # 100 MHz ticks -> us
        m = lambda v: np.median(v)   # noqa: E731
        print(f"n={n}: entry spread {m(a[:, 1] - a[:, 0]):.2f} us; first entry -> last partial row {m(a[:, 2] - a[:, 0]):.2f} us; "
              f"-> tail start {m(a[:, 3] - a[:, 0]):.2f} us; -> tail end {m(a[:, 4] - a[:, 0]):.2f} us", flush=True)


if __name__ == "__main__":
    main()
