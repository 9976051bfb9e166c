"""Acquisition value + gradient (``mpo_gp_acq_grad_host``, the polish objective) at
fixed points of fixed models: raw results saved per library (MPO_LIB_AB) to check
that a kernel change is bit-identical, and the wall time of one polish-sized round
(15 points, 1 thread).  Usage: acq_bits_probe.py OUT.npz [REF.npz]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd import _lib  # noqa: E402
from mpi_opt_amd.gp import DeviceGP  # noqa: E402
from oracle import gp_ei as O  # noqa: E402


def main():
    out = {}
    for n, d in [(57, 3), (96, 5), (256, 5), (448, 10), (700, 6)]:
        X, y = O.synthetic_problem(n, d, seed=n)
        rs = np.random.RandomState(d)
        gp = DeviceGP(X, y, amp=1.3, length_scale=rs.uniform(0.2, 1.5, d), noise=1e-4, device="cuda:0")
        P = rs.rand(15, d)
        codes = np.array([_lib.MPO_ACQ_EI, _lib.MPO_ACQ_PI, _lib.MPO_ACQ_LCB] * 5, dtype=np.int32)
        y_opt = float(np.min(y))
        f, g = gp.acq_grad(P, codes, y_opt)
        out[f"n{n}_f"], out[f"n{n}_g"] = f, g
        for _ in range(20):
            gp.acq_grad(P, codes, y_opt)
        R = 300
        t0 = time.perf_counter()
        for _ in range(R):
            gp.acq_grad(P, codes, y_opt)
        print(f"n={n}: {(time.perf_counter() - t0) / R * 1e6:.1f} us per 15-point round", flush=True)
    np.savez(sys.argv[1], **out)
    if len(sys.argv) > 2:
        ref = np.load(sys.argv[2])
        print("bit-identical:", all(np.array_equal(ref[k], out[k]) for k in out))


if __name__ == "__main__":
    main()
