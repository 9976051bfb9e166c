"""Same-box A/B runs: ``MPO_LIB_AB=ab_libs/<name>/libmpo.so`` makes a probe load
another revision's library (built by scripts/ab_libs.sh) instead of the in-tree
one.  Imported by the probes only; the product always loads
``mpi_opt_amd/libmpo.so``."""
import os

from mpi_opt_amd import _lib

if os.environ.get("MPO_LIB_AB"):
    if _lib._LIB is not None:
        raise RuntimeError("MPO_LIB_AB: libmpo.so was already loaded")
    _lib.LIB_PATH = os.path.abspath(os.environ["MPO_LIB_AB"])
