"""mpi_opt_amd -- MI355X-native engine for mpi_opt's trial-evaluation hot path.

Submodules are imported lazily so that CPU-only tooling (tests, the CLI parser)
can import the package without a GPU; every compute entry point goes through
``libmpo.so`` and raises if it is unavailable.
"""
__version__ = "0.1.0"
