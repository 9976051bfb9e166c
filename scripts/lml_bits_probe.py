"""Evaluate the device LML (+ gradient) of fixed problems / thetas and save the
raw results (npz): run once per library (MPO_LIB_AB) and compare the files to
check that a kernel change is bit-identical.  Usage: lml_bits_probe.py OUT.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd.gp_fit import DeviceLML, normalize_targets, theta_bounds  # noqa: E402
from oracle import gp_ei as O  # noqa: E402


def main():
    out = {}
    for n, d in [(57, 3), (96, 5), (130, 6), (256, 10), (500, 10)]:
        X, y = O.synthetic_problem(n, d, seed=n)
        dev = DeviceLML(X, normalize_targets(y)[0], device="cuda:0")
        b = theta_bounds(d)
        T = np.random.RandomState(d).uniform(b[:, 0], b[:, 1], size=(6, d + 2))
        T[0] = 0.0
        lml, grad, info = dev.evaluate(T)
        out[f"n{n}_lml"], out[f"n{n}_grad"], out[f"n{n}_info"] = lml, grad, info
        if n >= 256:   # a full group: the step kernel's tiles-per-wave > 1 path
            T40 = np.random.RandomState(d + 1).uniform(b[:, 0], b[:, 1], size=(40, d + 2))
            lml, grad, info = dev.evaluate(T40)
            out[f"n{n}_b40_lml"], out[f"n{n}_b40_grad"], out[f"n{n}_b40_info"] = lml, grad, info
    np.savez(sys.argv[1], **out)
    if len(sys.argv) > 2:
        ref = np.load(sys.argv[2])
        same = all(np.array_equal(ref[k], out[k]) for k in out)
        worst = max(float(np.nanmax(np.abs(ref[k] - out[k]) / np.maximum(np.abs(ref[k]), 1e-300)))
                    for k in out if not k.endswith("info"))
        print("bit-identical:", same, " max relative difference: %.3g" % worst)


if __name__ == "__main__":
    main()
