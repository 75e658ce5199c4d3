"""ctypes binding of libdrephip.so (include/drephip.h).

There is no fallback: if the HIP library is missing or cannot be loaded, every
entry point raises :class:`DrepHipError`.  Build it with
``python -c "import __graft_entry__ as g; g.build()"`` or ``make -C drep_amd/csrc``.

The library is linked against the HIP runtime (libamdhip64.so.7).  PyTorch-ROCm
ships its own copy; to keep exactly one HIP runtime in a process that may also
import torch (bench.py, the multi-GPU path), the torch copy is preloaded with
RTLD_GLOBAL before libdrephip.so when torch is installed, so both bind to it.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os
import sys
import threading
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DREPHIP_LIB", os.path.join(_HERE, "lib", "libdrephip.so"))

ERR = {0: "OK", -1: "invalid argument", -2: "HIP error", -3: "I/O error", -4: "out of memory",
       -5: "unsupported", -6: "internal error"}


class DrepHipError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()

u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
vp = C.c_void_p

# name -> (restype, argtypes); every symbol declared in include/drephip.h
SIGNATURES = {
    "drephip_version": (C.c_int, []),
    "drephip_build_id": (C.c_char_p, []),
    "drephip_last_error": (C.c_char_p, []),
    "drephip_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "drephip_create": (C.c_int, [C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.POINTER(vp)]),
    "drephip_destroy": (C.c_int, [vp]),
    "drephip_max_sketch": (C.c_uint32, []),
    "drephip_tile_bases": (C.c_uint64, []),
    "drephip_padded_bases": (C.c_uint64, [u64p, C.c_uint32]),
    "drephip_fasta_info": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "drephip_fasta_pack": (C.c_int, [C.c_char_p, C.c_int, u32p, u32p, C.c_uint64, C.c_uint64,
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "drephip_sketch": (C.c_int, [vp, u8p, u64p, C.c_uint32, u64p, C.c_uint32, u64p, u32p, u64p]),
    "drephip_sketch_files": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, C.c_int, u64p, u32p, u64p]),
    "drephip_last_ingest_stats": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                            C.POINTER(C.c_double), C.POINTER(C.c_uint32)]),
    "drephip_last_ingest_phases": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                             C.POINTER(C.c_uint32)]),
    "drephip_sketch_device": (C.c_int, [vp, vp, vp, u64p, u64p, u64p, C.c_uint32, vp, vp, vp]),
    "drephip_sketch_device_async": (C.c_int, [vp, vp, vp, u64p, u64p, u64p, C.c_uint32, vp, vp, vp]),
    "drephip_sketch_wait": (C.c_int, [vp, C.POINTER(C.c_int)]),
    "drephip_synth_device": (C.c_int, [vp, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                       vp, vp, vp]),
    "drephip_allpairs": (C.c_int, [vp, u64p, u32p, C.c_uint32, u16p, vp]),
    "drephip_allpairs_rows": (C.c_int, [vp, u64p, u32p, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp]),
    "drephip_allpairs_device": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp]),
    "drephip_allpairs_device_async": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp]),
    "drephip_allpairs_wait": (C.c_int, [vp]),
    "drephip_screen_geometry": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
    "drephip_screen_part": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), vp]),
    "drephip_screen_part_copy": (C.c_int, [vp, vp, vp, vp]),
    "drephip_screen_worth": (C.c_int, [vp, C.c_uint32, C.c_uint64, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "drephip_allpairs_device_marked": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp,
                                                 C.c_uint64, vp, C.c_uint64, vp]),
    "drephip_allpairs_merge_device": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp]),
    "drephip_distance_lut": (C.c_int, [C.c_int, C.c_uint32, f64p]),
    "drephip_write_mash_table": (C.c_int, [C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32, vp, vp, C.c_uint32,
                                           vp, vp, u16p, f64p, C.c_int]),
    "drephip_set_allpairs_path": (C.c_int, [vp, C.c_int, C.c_uint32]),
    "drephip_linkage": (C.c_int, [vp, f64p, C.c_uint32, C.c_int, f64p]),
    "drephip_linkage_counts_device": (C.c_int, [vp, vp, vp, C.c_uint32, u32p, f64p, C.c_uint32,
                                                np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS"),
                                                C.c_int, f64p, vp]),
    "drephip_linkage_square": (C.c_int, [vp, np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS"),
                                         C.c_uint32, C.c_int, f64p]),
    "drephip_mdb_square": (C.c_int, [C.c_uint32, vp, vp, C.c_uint32, vp, C.c_uint32, vp, vp, C.c_int, vp, vp, vp,
                                     vp, C.c_int]),
    "drephip_pivot_scan": (C.c_int, [C.c_uint64, vp, vp, C.c_int, C.c_uint32, u8p, u8p, C.POINTER(C.c_uint64),
                                     C.c_int]),
    "drephip_pivot_fill": (C.c_int, [C.c_uint64, vp, vp, C.c_int, vp, vp, C.c_uint32, vp, C.c_uint32, C.c_uint32,
                                     C.c_uint64, vp, C.c_int]),
    "drephip_linkage_reserve": (C.c_int, [vp, C.c_uint32]),
    "drephip_set_linkage_path": (C.c_int, [vp, C.c_int]),
    "drephip_linkage_sparse": (C.c_int, [C.c_uint32, C.c_uint64, u32p, u32p, f64p, C.c_int, f64p]),
    "drephip_last_linkage_info": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                            C.POINTER(C.c_uint32)]),
    "drephip_last_linkage_stats": (C.c_int, [vp] + [C.POINTER(C.c_double)] * 5),
    "drephip_last_linkage_launches": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
    "drephip_set_timing": (C.c_int, [vp, C.c_int]),
    "drephip_last_kernel_ms": (C.c_int, [vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "drephip_set_allpairs_screen": (C.c_int, [vp, C.c_int]),
    "drephip_last_screen_stats": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                             C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
}


def _preload_torch_hip_runtime() -> None:
    if "torch" in sys.modules:
        return  # torch already put its runtime in the process
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return
    for root in spec.submodule_search_locations:
        cand = os.path.join(root, "lib", "libamdhip64.so")
        if os.path.exists(cand):
            try:
                C.CDLL(cand, mode=C.RTLD_GLOBAL)
            except OSError:
                pass
            return


def lib():
    """Load libdrephip.so (once).  Raises DrepHipError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DrepHipError(
                "libdrephip.so not found at %s -- build it (make -C drep_amd/csrc); "
                "drep_amd has no CPU fallback" % LIB_PATH)
        _preload_torch_hip_runtime()
        try:
            L = C.CDLL(LIB_PATH)
        except OSError as e:
            raise DrepHipError("cannot load %s: %s" % (LIB_PATH, e)) from e
        for name, (res, args) in SIGNATURES.items():
            # an older build loaded for a same-box A/B (DREPHIP_LIB) may lack
            # entry points added since; the product library has them all
            # (tests/test_host.py checks the export list)
            if "DREPHIP_LIB" in os.environ and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        return L


def source_digest(root: Optional[str] = None) -> str:
    """sha256 of the library's sources as drep_amd/csrc/Makefile computes it
    for drephip_build_id: the `sha256sum` listing of include/drephip.h and the
    sorted drep_amd/csrc/*.{cpp,h,hip} + Makefile, hashed again."""
    import glob
    import hashlib
    root = root or os.path.dirname(_HERE)
    csrc = os.path.join(root, "drep_amd", "csrc")
    names = sorted([os.path.basename(p) for ext in ("*.hip", "*.cpp", "*.h")
                    for p in glob.glob(os.path.join(csrc, ext))] + ["Makefile"])
    files = ["include/drephip.h"] + ["drep_amd/csrc/" + n for n in names]
    listing = "".join("%s  %s\n" % (hashlib.sha256(open(os.path.join(root, f), "rb").read()).hexdigest(), f)
                      for f in files)
    return hashlib.sha256(listing.encode()).hexdigest()


def build_id() -> dict:
    """The loaded library's build identity (drephip_build_id) as a dict."""
    raw = lib().drephip_build_id().decode()
    return dict(kv.split("=", 1) for kv in raw.split(";") if "=" in kv)


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().drephip_last_error().decode("utf-8", "replace")
        raise DrepHipError("%s failed (%s): %s" % (what, ERR.get(rc, rc), msg))


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().drephip_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def max_sketch() -> int:
    """Largest supported sketch size s."""
    return int(lib().drephip_max_sketch())


def tile_bases() -> int:
    return int(lib().drephip_tile_bases())


def padded_bases(rec_len: Sequence[int]) -> int:
    a = np.ascontiguousarray(rec_len, dtype=np.uint64)
    return int(lib().drephip_padded_bases(a if len(a) else np.zeros(1, np.uint64), len(a)))


def distance_lut(denom: int, k: int = 21) -> np.ndarray:
    out = np.zeros(denom + 1, dtype=np.float64)
    check(lib().drephip_distance_lut(k, denom, out), "drephip_distance_lut")
    return out


def write_mash_table(path: str, names: Sequence[str], common: np.ndarray, denom: Optional[np.ndarray], s: int,
                     dist: np.ndarray, pval: np.ndarray, self_count: np.ndarray, self_pval: np.ndarray,
                     threads: int = 0) -> None:
    """drephip_write_mash_table: condensed arrays (i < j), names of the N genomes."""
    N = len(names)
    npairs = N * (N - 1) // 2
    common = np.ascontiguousarray(common, dtype=np.uint16)
    dist = np.ascontiguousarray(dist, dtype=np.float64)
    pval = np.ascontiguousarray(pval, dtype=np.float64)
    for a in (common, dist, pval) + ((denom,) if denom is not None else ()):
        if len(a) != npairs:
            raise ValueError("condensed arrays must hold N(N-1)/2 = %d entries" % npairs)
    den = None if denom is None else np.ascontiguousarray(denom, dtype=np.uint16)
    arr = (C.c_char_p * max(N, 1))(*[os.fsencode(n) for n in names])
    check(lib().drephip_write_mash_table(os.fsencode(path), arr, N, common.ctypes.data,
                                         None if den is None else den.ctypes.data, int(s), dist.ctypes.data,
                                         pval.ctypes.data, np.ascontiguousarray(self_count, dtype=np.uint16),
                                         np.ascontiguousarray(self_pval, dtype=np.float64), int(threads)),
          "drephip_write_mash_table(%s)" % path)


def fasta_info(path: str, k: int = 21):
    length = C.c_uint64(0)
    padded = C.c_uint64(0)
    nrec = C.c_uint32(0)
    nk = C.c_uint64(0)
    check(lib().drephip_fasta_info(path.encode(), k, C.byref(length), C.byref(padded), C.byref(nrec),
                                   C.byref(nk)), "drephip_fasta_info(%s)" % path)
    return {"length": length.value, "padded": padded.value, "n_records": nrec.value, "n_kmers": nk.value}


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


def mdb_square(N: int, common: np.ndarray, denom: Optional[np.ndarray], s: int, lut32: np.ndarray,
               lut_off: np.ndarray, codes: np.ndarray, threads: int = 0, want_sim: bool = True):
    """drephip_mdb_square (host): the N^2-row Mdb columns from the condensed
    counts -- (g1 codes, g2 codes, dist, similarity) in all_vs_all_MASH's row
    order; codes' dtype (int8/16/32) is the category code width."""
    common = np.ascontiguousarray(common, dtype=np.uint16)
    den = None if denom is None else np.ascontiguousarray(denom, dtype=np.uint16)
    lut32 = np.ascontiguousarray(lut32, dtype=np.float32)
    lut_off = np.ascontiguousarray(lut_off, dtype=np.int32)
    codes = np.ascontiguousarray(codes)
    if codes.dtype not in (np.int8, np.int16, np.int32) or len(codes) != N or len(lut_off) != s + 1:
        raise ValueError("codes must be N int8/int16/int32 category codes and lut_off s+1 offsets")
    npairs = N * (N - 1) // 2
    if len(common) != npairs or (den is not None and len(den) != npairs):
        raise ValueError("condensed arrays must hold N(N-1)/2 = %d entries" % npairs)
    codes32 = codes.astype(np.int32)
    g1 = np.empty(N * N, dtype=codes.dtype)
    g2 = np.empty(N * N, dtype=codes.dtype)
    dist = np.empty(N * N, dtype=np.float32)
    sim = np.empty(N * N, dtype=np.float32) if want_sim else None
    check(lib().drephip_mdb_square(N, _ptr(common) if npairs else None, _ptr(den) if npairs else None, int(s),
                                   _ptr(lut32), len(lut32), _ptr(lut_off), _ptr(codes32), codes.dtype.itemsize,
                                   _ptr(g1), _ptr(g2), _ptr(dist), _ptr(sim), int(threads)), "drephip_mdb_square")
    return g1, g2, dist, sim


def pivot_scan(codes1: np.ndarray, codes2: np.ndarray, ncat: int, threads: int = 0):
    """drephip_pivot_scan: (present1, present2, period) of two category-code
    columns; raises DrepHipError(-5) on a missing (negative) code."""
    codes1 = np.ascontiguousarray(codes1)
    codes2 = np.ascontiguousarray(codes2)
    if codes1.dtype != codes2.dtype or codes1.dtype not in (np.int8, np.int16, np.int32) or len(codes1) != len(codes2):
        raise ValueError("codes1/codes2 must be equal-length int8/int16/int32 arrays")
    p1 = np.zeros(max(ncat, 1), np.uint8)
    p2 = np.zeros(max(ncat, 1), np.uint8)
    period = C.c_uint64(0)
    check(lib().drephip_pivot_scan(len(codes1), _ptr(codes1), _ptr(codes2), codes1.dtype.itemsize, int(ncat), p1, p2,
                                   C.byref(period), int(threads)), "drephip_pivot_scan")
    return p1[:ncat].astype(bool), p2[:ncat].astype(bool), int(period.value)


def pivot_fill(codes1: np.ndarray, codes2: np.ndarray, pos1: np.ndarray, pos2: np.ndarray, vals: np.ndarray,
               n1: int, n2: int, period: int = 0, threads: int = 0) -> np.ndarray:
    """drephip_pivot_fill: the n1 x n2 float32 pivot of `vals`; raises
    DrepHipError(-1, "Index contains duplicate entries...") like pandas."""
    codes1 = np.ascontiguousarray(codes1)
    codes2 = np.ascontiguousarray(codes2)
    pos1 = np.ascontiguousarray(pos1, dtype=np.int32)
    pos2 = np.ascontiguousarray(pos2, dtype=np.int32)
    vals = np.ascontiguousarray(vals, dtype=np.float32)
    if not (len(codes1) == len(codes2) == len(vals)) or len(pos1) != len(pos2):
        raise ValueError("codes/vals lengths or pos lengths differ")
    out = np.empty((n1, n2), dtype=np.float32)
    check(lib().drephip_pivot_fill(len(vals), _ptr(codes1), _ptr(codes2), codes1.dtype.itemsize, _ptr(pos1), _ptr(pos2),
                                   len(pos1), _ptr(vals), int(n1), int(n2), int(period), _ptr(out), int(threads)),
          "drephip_pivot_fill")
    return out


# scipy linkage method codes (include/drephip.h DREPHIP_LINK_*)
LINK_METHODS = {"single": 0, "complete": 1, "average": 2, "weighted": 6}


def linkage_sparse(n: int, i: np.ndarray, j: np.ndarray, v: np.ndarray, method: str) -> np.ndarray:
    """drephip_linkage_sparse (host only, no GPU): scipy's linkage Z of the n x n
    distance matrix that holds v[t] at (i[t], j[t]) and 1.0 at every pair not
    listed (each unordered pair at most once, v in [0, 1))."""
    i = np.ascontiguousarray(i, dtype=np.uint32)
    j = np.ascontiguousarray(j, dtype=np.uint32)
    v = np.ascontiguousarray(v, dtype=np.float64)
    if not (len(i) == len(j) == len(v)):
        raise ValueError("i, j and v must have one entry per pair")
    Z = np.zeros((max(n - 1, 0), 4), dtype=np.float64)
    if n >= 2:
        e = np.zeros(1, np.uint32)
        check(lib().drephip_linkage_sparse(int(n), len(v), i if len(i) else e, j if len(j) else e,
                                           v if len(v) else np.zeros(1), LINK_METHODS[method], Z.reshape(-1)),
              "drephip_linkage_sparse")
    return Z


class Context:
    """One libdrephip context: a HIP device plus (k, s, seed)."""

    def __init__(self, device: int = 0, k: int = 21, s: int = 1000, seed: int = 42):
        L = lib()
        self.k, self.s, self.seed, self.device = int(k), int(s), int(seed), int(device)
        h = vp()
        check(L.drephip_create(self.device, self.k, self.s, self.seed, C.byref(h)), "drephip_create")
        self._h = h

    # -- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().drephip_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # all-pairs kernel selection (include/drephip.h DREPHIP_AP_*)
    AP_AUTO, AP_TABLE, AP_BAND, AP_MERGE = 0, 1, 2, 3

    SCREEN_AUTO, SCREEN_ON, SCREEN_OFF = 0, 1, 2

    def set_allpairs_screen(self, mode: int) -> None:
        """The shared-hash screen in front of the all-pairs kernels
        (include/drephip.h: auto / on / off)."""
        check(lib().drephip_set_allpairs_screen(self._h, mode), "drephip_set_allpairs_screen")
        self._screen_mode = mode

    @property
    def allpairs_screen(self) -> int:
        return getattr(self, "_screen_mode", self.SCREEN_AUTO)

    def screen_stats(self) -> dict:
        u = C.c_int(0)
        e, r, c, m, sp = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        check(lib().drephip_last_screen_stats(self._h, C.byref(u), C.byref(e), C.byref(r), C.byref(c), C.byref(m),
                                              C.byref(sp)), "drephip_last_screen_stats")
        return {"used": bool(u.value), "entries": e.value, "runs": r.value, "checks": c.value, "marked": m.value,
                "simple": sp.value}

    def set_allpairs_path(self, path: int, band_cap: int = 1024) -> None:
        check(lib().drephip_set_allpairs_path(self._h, path, band_cap), "drephip_set_allpairs_path")

    LINK_METHODS = LINK_METHODS
    # linkage path (include/drephip.h DREPHIP_LINK_PATH_*)
    LINK_AUTO, LINK_DENSE, LINK_SPARSE = 0, 1, 2

    def set_linkage_path(self, path: int) -> None:
        check(lib().drephip_set_linkage_path(self._h, int(path)), "drephip_set_linkage_path")

    def linkage_info(self):
        """{sparse, pairs, components, largest} of the last linkage call."""
        sp, npairs, nc, lg = C.c_int(0), C.c_uint64(0), C.c_uint32(0), C.c_uint32(0)
        check(lib().drephip_last_linkage_info(self._h, C.byref(sp), C.byref(npairs), C.byref(nc), C.byref(lg)),
              "drephip_last_linkage_info")
        return {"sparse": bool(sp.value), "pairs": npairs.value, "components": nc.value, "largest": lg.value}

    def linkage(self, y: np.ndarray, method: str) -> np.ndarray:
        """scipy.cluster.hierarchy.linkage(y, method) on the GPU, bit-identical
        (y: condensed float64 distances)."""
        y = np.ascontiguousarray(y, dtype=np.float64)
        n = int(round((1 + (1 + 8 * len(y)) ** 0.5) / 2))
        if n * (n - 1) // 2 != len(y):
            raise ValueError("y is not a condensed distance vector")
        Z = np.zeros((max(n - 1, 0), 4), dtype=np.float64)
        if n >= 2:
            check(lib().drephip_linkage(self._h, y, n, self.LINK_METHODS[method], Z.reshape(-1)),
                  "drephip_linkage")
        return Z

    def linkage_square(self, M: np.ndarray, method: str) -> np.ndarray:
        """scipy.cluster.hierarchy.linkage(squareform(M), method) on the GPU,
        bit-identical, with squareform's and linkage's checks (DrepHipError
        carrying scipy's message when one fails); M: n x n float32."""
        M = np.ascontiguousarray(M, dtype=np.float32)
        if M.ndim != 2 or M.shape[0] != M.shape[1]:
            raise ValueError("M must be a square matrix")
        n = M.shape[0]
        Z = np.zeros((max(n - 1, 0), 4), dtype=np.float64)
        if n >= 2:
            check(lib().drephip_linkage_square(self._h, M, n, self.LINK_METHODS[method], Z.reshape(-1)),
                  "drephip_linkage_square")
        return Z

    def linkage_counts_device(self, d_common: int, d_denom: Optional[int], n: int, perm: np.ndarray,
                              lut: np.ndarray, lut_off: np.ndarray, method: str,
                              stream: Optional[int] = None) -> np.ndarray:
        """linkage() of the distances given by device-resident all-pairs counts
        (see drephip_linkage_counts_device); the counts are read after the work
        queued on `stream`."""
        Z = np.zeros((max(n - 1, 0), 4), dtype=np.float64)
        if n >= 2:
            check(lib().drephip_linkage_counts_device(
                self._h, d_common, d_denom, n, np.ascontiguousarray(perm, dtype=np.uint32),
                np.ascontiguousarray(lut, dtype=np.float64), len(lut),
                np.ascontiguousarray(lut_off, dtype=np.int32), self.LINK_METHODS[method], Z.reshape(-1), stream),
                "drephip_linkage_counts_device")
        return Z

    def linkage_reserve(self, n: int) -> None:
        """Allocate the n x n linkage matrix now (drephip_linkage_reserve)."""
        check(lib().drephip_linkage_reserve(self._h, int(n)), "drephip_linkage_reserve")

    def linkage_stats(self):
        """{alloc_s, matrix_s, chain_s, finish_s, wall_s} of the last linkage call."""
        v = [C.c_double(0) for _ in range(5)]
        check(lib().drephip_last_linkage_stats(self._h, *[C.byref(x) for x in v]), "drephip_last_linkage_stats")
        return dict(zip(("alloc_s", "matrix_s", "chain_s", "finish_s", "wall_s"), (x.value for x in v)))

    def linkage_launches(self) -> int:
        """Step launches of the last dense-chain linkage call."""
        v = C.c_uint64(0)
        check(lib().drephip_last_linkage_launches(self._h, C.byref(v)), "drephip_last_linkage_launches")
        return int(v.value)

    def set_timing(self, on: bool = True, kernels=None) -> None:
        """HIP-event timing of kernel launches: all kernels, or only the
        `which` indices in `kernels` (see kernel_ms)."""
        mask = 0 if not on else (-1 if kernels is None else sum(1 << int(w) for w in kernels))
        check(lib().drephip_set_timing(self._h, mask), "drephip_set_timing")

    def kernel_ms(self, which: int):
        ms = C.c_double(0)
        n = C.c_int(0)
        check(lib().drephip_last_kernel_ms(self._h, which, C.byref(ms), C.byref(n)), "drephip_last_kernel_ms")
        return ms.value, n.value

    # -- sketch
    def sketch_files(self, paths: Sequence[str], threads: int = 0):
        n = len(paths)
        hashes = np.zeros((n, self.s), dtype=np.uint64)
        nhash = np.zeros(n, dtype=np.uint32)
        length = np.zeros(n, dtype=np.uint64)
        if n == 0:
            return hashes, nhash, length
        arr = (C.c_char_p * n)(*[os.fsencode(p) for p in paths])
        check(lib().drephip_sketch_files(self._h, arr, n, int(threads), hashes.reshape(-1), nhash, length),
              "drephip_sketch_files")
        return hashes, nhash, length

    def ingest_stats(self):
        """{produce_s, gpu_s, wall_s, batches} of the last sketch_files call."""
        a, b, c = C.c_double(0), C.c_double(0), C.c_double(0)
        n = C.c_uint32(0)
        check(lib().drephip_last_ingest_stats(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(n)),
              "drephip_last_ingest_stats")
        r, p = C.c_double(0), C.c_double(0)
        o = C.c_uint32(0)
        check(lib().drephip_last_ingest_phases(self._h, C.byref(r), C.byref(p), C.byref(o)),
              "drephip_last_ingest_phases")
        return {"produce_s": a.value, "gpu_s": b.value, "wall_s": c.value, "batches": n.value,
                "read_thread_s": r.value, "pack_thread_s": p.value, "overflow_genomes": o.value}

    def sketch_records(self, seq: np.ndarray, rec_off: np.ndarray, genome_rec_off: np.ndarray):
        seq = np.ascontiguousarray(seq, dtype=np.uint8)
        rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
        genome_rec_off = np.ascontiguousarray(genome_rec_off, dtype=np.uint64)
        n = len(genome_rec_off) - 1
        hashes = np.zeros((max(n, 0), self.s), dtype=np.uint64)
        nhash = np.zeros(max(n, 0), dtype=np.uint32)
        length = np.zeros(max(n, 0), dtype=np.uint64)
        if n <= 0:
            return hashes, nhash, length
        check(lib().drephip_sketch(self._h, seq if len(seq) else np.zeros(1, np.uint8), rec_off,
                                   len(rec_off) - 1, genome_rec_off, n, hashes.reshape(-1), nhash, length),
              "drephip_sketch")
        return hashes, nhash, length

    def sketch_device(self, d_codes: int, d_valid: int, base_off, padded, nkmers, n: int,
                      d_hashes: int, d_nhash: int, stream: Optional[int] = None) -> None:
        check(lib().drephip_sketch_device(self._h, d_codes, d_valid,
                                          np.ascontiguousarray(base_off, dtype=np.uint64),
                                          np.ascontiguousarray(padded, dtype=np.uint64),
                                          np.ascontiguousarray(nkmers, dtype=np.uint64), n,
                                          d_hashes, d_nhash, stream), "drephip_sketch_device")

    def sketch_device_async(self, d_codes: int, d_valid: int, base_off, padded, nkmers, n: int,
                            d_hashes: int, d_nhash: int, stream: Optional[int] = None) -> None:
        """sketch_device without the wait: the sketches are final after
        sketch_wait() (include/drephip.h)."""
        check(lib().drephip_sketch_device_async(self._h, d_codes, d_valid,
                                                np.ascontiguousarray(base_off, dtype=np.uint64),
                                                np.ascontiguousarray(padded, dtype=np.uint64),
                                                np.ascontiguousarray(nkmers, dtype=np.uint64), n,
                                                d_hashes, d_nhash, stream), "drephip_sketch_device_async")

    def sketch_wait(self) -> bool:
        """Completes sketch_device_async; True if the sketches were recomputed
        (results derived from them in between must be recomputed)."""
        redone = C.c_int(0)
        check(lib().drephip_sketch_wait(self._h, C.byref(redone)), "drephip_sketch_wait")
        return bool(redone.value)

    def synth_device(self, seed: int, g0: int, n: int, family_size: int, L: int, d_codes: int,
                     d_valid: int, stream: Optional[int] = None) -> None:
        check(lib().drephip_synth_device(self._h, seed, g0, n, family_size, L, d_codes, d_valid, stream),
              "drephip_synth_device")

    # -- all-pairs
    def allpairs(self, hashes: np.ndarray, nhash: np.ndarray, want_denom: Optional[bool] = None):
        hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
        nhash = np.ascontiguousarray(nhash, dtype=np.uint32)
        N = len(nhash)
        if hashes.shape != (N, self.s):
            raise ValueError("hashes must be [N, s] = [%d, %d], got %s" % (N, self.s, hashes.shape))
        npairs = N * (N - 1) // 2
        if want_denom is None:
            want_denom = bool((nhash < self.s).any())
        common = np.zeros(max(npairs, 1), dtype=np.uint16)
        denom = np.zeros(max(npairs, 1), dtype=np.uint16) if want_denom else None
        if N >= 2:
            check(lib().drephip_allpairs(self._h, hashes.reshape(-1), nhash, N, common,
                                         denom.ctypes.data if denom is not None else None),
                  "drephip_allpairs")
        common = common[:npairs]
        if denom is None:
            denom = np.full(npairs, self.s, dtype=np.uint16)
        else:
            denom = denom[:npairs]
        return common, denom

    def allpairs_rows(self, hashes: np.ndarray, nhash: np.ndarray, row0: int, row1: int,
                      common_out: np.ndarray, denom_out: Optional[np.ndarray] = None) -> None:
        """Rows [row0, row1) of the triangle into the given condensed segment
        views (uint16, contiguous; length = pairs of those rows)."""
        hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
        nhash = np.ascontiguousarray(nhash, dtype=np.uint32)
        N = len(nhash)
        if hashes.shape != (N, self.s):
            raise ValueError("hashes must be [N, s] = [%d, %d], got %s" % (N, self.s, hashes.shape))
        r1 = min(row1, N - 1)

        def start(i):
            return i * N - i * (i + 1) // 2
        n = max(0, start(r1) - start(row0)) if row0 < r1 else 0
        for arr in (common_out, denom_out):
            if arr is not None and (arr.dtype != np.uint16 or not arr.flags.c_contiguous or len(arr) < n):
                raise ValueError("segment buffers must be contiguous uint16 of length >= %d" % n)
        if n == 0:
            return
        check(lib().drephip_allpairs_rows(self._h, hashes.reshape(-1), nhash, N, row0, row1,
                                          common_out.ctypes.data,
                                          denom_out.ctypes.data if denom_out is not None else None),
              "drephip_allpairs_rows")

    def allpairs_device(self, d_hashes: int, d_nhash: int, N: int, row0: int, row1: int, d_common: int,
                        d_denom: Optional[int] = None, stream: Optional[int] = None, merge: bool = False):
        fn = lib().drephip_allpairs_merge_device if merge else lib().drephip_allpairs_device
        check(fn(self._h, d_hashes, d_nhash, N, row0, row1, d_common, d_denom, stream),
              "drephip_allpairs_device")

    # ---- the sharded screen (include/drephip.h: drephip_screen_part ...)
    def screen_geometry(self) -> int:
        """Rows per row tile of the sharded screen's marks (tile T = rows [T R, (T + 1) R))."""
        r = C.c_uint32()
        check(lib().drephip_screen_geometry(self._h, C.byref(r)), "drephip_screen_geometry")
        return r.value

    def screen_part(self, d_hashes: int, d_nhash: int, N: int, part: int, nparts: int,
                    stream: Optional[int] = None) -> Tuple[int, int, int]:
        """Group hash part `part` of `nparts`: (its pair checks, its cell words, its records)."""
        c, nc, n = C.c_uint64(), C.c_uint32(), C.c_uint32()
        check(lib().drephip_screen_part(self._h, d_hashes, d_nhash, N, part, nparts, C.byref(c), C.byref(nc),
                                        C.byref(n), stream), "drephip_screen_part")
        return c.value, nc.value, n.value

    def screen_part_copy(self, d_cells: Optional[int], d_records: Optional[int], stream: Optional[int] = None) -> None:
        check(lib().drephip_screen_part_copy(self._h, d_cells, d_records, stream), "drephip_screen_part_copy")

    def screen_worth(self, N: int, checks: int) -> Tuple[bool, bool]:
        """(the screen applies to N genomes at all, it would run with these checks)."""
        a, u = C.c_int(), C.c_int()
        check(lib().drephip_screen_worth(self._h, N, checks, C.byref(a), C.byref(u)), "drephip_screen_worth")
        return bool(a.value), bool(u.value)

    def allpairs_device_marked(self, d_hashes: int, d_nhash: int, N: int, row0: int, row1: int, d_common: int,
                               d_denom: Optional[int], d_cells: Optional[int], n_cells: int, d_records: Optional[int],
                               n_records: int, stream: Optional[int] = None) -> None:
        check(lib().drephip_allpairs_device_marked(self._h, d_hashes, d_nhash, N, row0, row1, d_common, d_denom,
                                                   d_cells, n_cells, d_records, n_records, stream),
              "drephip_allpairs_device_marked")

    def allpairs_device_async(self, d_hashes: int, d_nhash: int, N: int, row0: int, row1: int,
                              d_common: int, d_denom: Optional[int] = None, stream: Optional[int] = None):
        """allpairs_device whose failure-count check is deferred to
        allpairs_wait() (include/drephip.h)."""
        check(lib().drephip_allpairs_device_async(self._h, d_hashes, d_nhash, N, row0, row1, d_common,
                                                  d_denom, stream), "drephip_allpairs_device_async")

    def allpairs_wait(self) -> None:
        check(lib().drephip_allpairs_wait(self._h), "drephip_allpairs_wait")
