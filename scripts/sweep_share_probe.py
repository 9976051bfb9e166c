"""Share of the pivot sweeps in one LML launch of the fused split sweep: the launch
timed with HIP events as is and with MPO_FIT_DEBUG=23 (sw_step_kernel skips the
32x32 pivot sweep; results invalid, timing of everything else)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import _lib, synthetic  # noqa: E402
from mpi_opt_amd.gp_fit import DeviceLML, normalize_targets  # noqa: E402


def kernel_us(dev, T, reps=50):
    dev.evaluate(T)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        _lib.check(_lib.lib().mpo_gp_lml_grad(
            _lib.ptr(dev.X), _lib.ptr(dev.y), dev.n, dev.d, _lib.ptr(dev.theta_d), T.shape[0], _lib.ptr(dev.lml_d),
            _lib.ptr(dev.grad_d), _lib.ptr(dev.info_d), _lib.ptr(dev.ws), dev.ws_bytes, s.cuda_stream))
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for n in (128, 256, 512):
    X, y = synthetic.gp_problem(n, 5, 0)
    dev = DeviceLML(X, normalize_targets(y)[0], device="cuda:0")
    T = np.zeros((3, 7))
    T[1] += 0.5
    T[2] -= 0.5
    os.environ.pop("MPO_FIT_DEBUG", None)
    full = kernel_us(dev, T)
    os.environ["MPO_FIT_DEBUG"] = "23"
    nosweep = kernel_us(dev, T)
    os.environ.pop("MPO_FIT_DEBUG")
    print(f"n={n}: LML launch {full:.1f} us, without the pivot sweeps {nosweep:.1f} us -> sweeps {full - nosweep:.1f} us "
          f"({(full - nosweep) / full:.0%})", flush=True)
