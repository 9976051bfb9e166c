"""Where concurrent refits saturate: T threads each (a) calling one LML round
(DeviceLML.evaluate, 3 thetas, n obs) in a loop -- the device + ctypes side --
and (b) driving scipy's L-BFGS-B (the lockstep driver) on a cheap host objective
-- the GIL-held side.  Rounds per second for each T."""
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd import gp_fit as GF  # noqa: E402


def run_threads(T, fn, seconds=1.5):
    counts = [0] * T
    stop = time.perf_counter() + seconds

    def work(i):
        torch.cuda.set_device(0)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            state = fn(i, None)
            while time.perf_counter() < stop:
                fn(i, state)
                counts[i] += 1

    ths = [threading.Thread(target=work, args=(i,)) for i in range(T)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return sum(counts) / (time.perf_counter() - t0)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    d = 5
    rng = np.random.RandomState(0)
    X = rng.rand(n, d)
    y = np.sin(X @ rng.randn(d))
    yn, _, _ = GF.normalize_targets(y)
    th = np.zeros((3, d + 2))

    def lml_round(i, st):
        if st is None:
            st = GF.DeviceLML(X, yn, device="cuda:0")
            st.evaluate(th)
            return st
        st.evaluate(th)

    def host_fit(i, st):
        if st is None:
            return True
        # the lockstep driver on a quadratic objective: host work per round only
        def ev(T_):
            T_ = np.asarray(T_)
            return -np.sum((T_ - 0.3) ** 2, axis=1), -2 * (T_ - 0.3), np.zeros(len(T_), np.int32)
        GF.lockstep_lbfgsb(ev, d, i, 2, False)

    for T in (1, 2, 4, 8):
        r = run_threads(T, lml_round)
        print(f"n={n} T={T}: LML rounds (device + ctypes) {r:8.0f} /s", flush=True)
    for T in (1, 2, 4, 8):
        t0 = time.perf_counter()
        r = run_threads(T, host_fit)
        print(f"T={T}: host L-BFGS-B fits on a quadratic {r:8.1f} /s", flush=True)
    # rounds per quadratic fit, for scale
    cnt = [0]

    def ev2(T_):
        cnt[0] += 1
        T_ = np.asarray(T_)
        return -np.sum((T_ - 0.3) ** 2, axis=1), -2 * (T_ - 0.3), np.zeros(len(T_), np.int32)
    GF.lockstep_lbfgsb(ev2, d, 0, 2, False)
    print(f"rounds per quadratic fit: {cnt[0]}")


if __name__ == "__main__":
    main()
