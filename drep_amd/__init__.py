"""drep_amd -- MI355X-native drop-in for dRep's primary-clustering Mash step.

The reference (SilasK/drep, drep/d_cluster.py:481-630) shells out to the Mash
binary to sketch every genome and compute all-vs-all Mash distances, then
clusters the resulting Mdb table with scipy.  This package keeps that Python
surface (``d_cluster.all_vs_all_MASH`` -> Mdb, ``cluster_mash_database`` ->
Cdb) and runs the sketch and all-pairs arithmetic in hand-written HIP kernels
for gfx950 (libdrephip.so, C ABI in include/drephip.h).  There is no CPU
fallback: without the HIP library every compute call raises.
"""
from . import mash_io
from ._lib import Context, DrepHipError

__all__ = ["Context", "DrepHipError", "mash_io", "d_cluster"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "d_cluster":   # lazy: pulls in pandas/scipy
        import importlib
        return importlib.import_module(".d_cluster", __name__)
    raise AttributeError(name)
