"""ctypes binding of the CPU oracle (oracle/mash_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package ``drep_amd``.
It restates Mash's sketch/dist arithmetic (Mash itself is a third-party binary
absent from /root/reference; see the header of mash_oracle.c) and is pinned by
the reference fixtures copied to tests/golden/ (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        L.oracle_murmur3_h1.restype = C.c_uint64
        L.oracle_murmur3_h1.argtypes = [C.c_char_p, C.c_int, C.c_uint32]
        L.oracle_sketch_fasta.argtypes = [C.c_char_p, C.c_int, C.c_uint32, C.c_uint32,
                                          u64p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
        L.oracle_sketch_fasta_many.argtypes = [C.POINTER(C.c_char_p), C.c_uint32, C.c_int, C.c_uint32,
                                               C.c_uint32, u64p, u32p, u64p, C.c_int]
        L.oracle_sketch_records.argtypes = [u8p, u64p, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32,
                                            u64p, C.POINTER(C.c_uint32)]
        L.oracle_sketch_records_sortuniq.argtypes = L.oracle_sketch_records.argtypes
        L.oracle_synth_base.restype = C.c_uint32
        L.oracle_synth_base.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64]
        L.oracle_synth_ascii.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, u8p]
        L.oracle_sketch_synth.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                          C.c_int, C.c_uint32, C.c_uint32, u64p, u32p, C.c_int]
        L.oracle_dist_pair.argtypes = [u64p, C.c_uint32, u64p, C.c_uint32, C.c_uint32,
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.oracle_mash_distance.restype = C.c_double
        L.oracle_mash_distance.argtypes = [C.c_uint32, C.c_uint32, C.c_int]
        L.oracle_allpairs_rows.argtypes = [u64p, u32p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                           u16p, C.c_void_p, C.c_int]
        L.oracle_dist_pairs_list.argtypes = [u64p, u32p, C.c_uint32, u32p, u32p, C.c_uint64, u16p, C.c_int]
        L.oracle_max_threads.restype = C.c_int
        L.oracle_read_fasta.argtypes = [C.c_char_p, C.POINTER(C.POINTER(C.c_uint8)),
                                        C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


def murmur3_h1(data: bytes, seed: int = 42) -> int:
    return int(lib().oracle_murmur3_h1(data, len(data), seed))


def sketch_fasta(path: str, k: int = 21, s: int = 1000, seed: int = 42):
    out = np.zeros(s, dtype=np.uint64)
    n = C.c_uint32(0)
    length = C.c_uint64(0)
    rc = lib().oracle_sketch_fasta(path.encode(), k, s, seed, out, C.byref(n), C.byref(length))
    if rc != 0:
        raise OSError("oracle could not read %s" % path)
    return out[: n.value].copy(), int(length.value)


def sketch_fasta_many(paths, k=21, s=1000, seed=42, threads=0):
    n = len(paths)
    arr = (C.c_char_p * n)(*[p.encode() for p in paths])
    out = np.zeros((n, s), dtype=np.uint64)
    nh = np.zeros(n, dtype=np.uint32)
    ln = np.zeros(n, dtype=np.uint64)
    rc = lib().oracle_sketch_fasta_many(arr, n, k, s, seed, out.reshape(-1), nh, ln, threads)
    if rc != 0:
        raise OSError("oracle could not read one of the FASTAs")
    return out, nh, ln


def sketch_records(seq: np.ndarray, rec_off: np.ndarray, k=21, s=1000, seed=42, spec=False):
    """Sketch one genome given as upper-case ASCII records (rec_off has n+1 entries)."""
    seq = np.ascontiguousarray(seq, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    out = np.zeros(s, dtype=np.uint64)
    n = C.c_uint32(0)
    fn = lib().oracle_sketch_records_sortuniq if spec else lib().oracle_sketch_records
    fn(seq if len(seq) else np.zeros(1, np.uint8), rec_off, len(rec_off) - 1, k, s, seed, out, C.byref(n))
    return out[: n.value].copy()


def read_fasta(path: str):
    """(concatenated upper-case sequence bytes, record offsets, total length)."""
    L = lib()
    sp = C.POINTER(C.c_uint8)()
    op = C.POINTER(C.c_uint64)()
    nrec = C.c_uint32(0)
    ln = C.c_uint64(0)
    if L.oracle_read_fasta(path.encode(), C.byref(sp), C.byref(op), C.byref(nrec), C.byref(ln)) != 0:
        raise OSError(path)
    seq = np.ctypeslib.as_array(sp, shape=(max(ln.value, 1),))[: ln.value].copy()
    off = np.ctypeslib.as_array(op, shape=(nrec.value + 1,)).copy()
    libc = C.CDLL(None)
    libc.free(sp)
    libc.free(op)
    return seq, off, int(ln.value)


def synth_ascii(g: int, L: int, seed: int = 0, family_size: int = 100) -> np.ndarray:
    out = np.zeros(L, dtype=np.uint8)
    lib().oracle_synth_ascii(seed, g, family_size, L, out)
    return out


def sketch_synth(g0: int, n: int, L: int, seed: int = 0, family_size: int = 100,
                 k: int = 21, s: int = 1000, hseed: int = 42, threads: int = 0):
    out = np.zeros((n, s), dtype=np.uint64)
    nh = np.zeros(n, dtype=np.uint32)
    rc = lib().oracle_sketch_synth(seed, g0, n, family_size, L, k, s, hseed, out.reshape(-1), nh, threads)
    if rc != 0:
        raise MemoryError("oracle synthetic sketch failed")
    return out, nh


def dist_pair(a: np.ndarray, b: np.ndarray, s: int):
    c = C.c_uint32(0)
    d = C.c_uint32(0)
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    lib().oracle_dist_pair(a if len(a) else np.zeros(1, np.uint64), len(a),
                           b if len(b) else np.zeros(1, np.uint64), len(b), s, C.byref(c), C.byref(d))
    return int(c.value), int(d.value)


def mash_distance(common: int, denom: int, k: int = 21) -> float:
    return float(lib().oracle_mash_distance(common, denom, k))


def allpairs(hashes: np.ndarray, nhash: np.ndarray, s: int, r0: int = 0, r1=None,
             want_denom: bool = True, threads: int = 0):
    """Condensed (i<j, row-major) common / denom for rows [r0, r1)."""
    hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
    nhash = np.ascontiguousarray(nhash, dtype=np.uint32)
    N = len(nhash)
    r1 = N if r1 is None else r1

    def start(i):
        return i * N - i * (i + 1) // 2

    npairs = start(r1) - start(r0)
    common = np.zeros(max(npairs, 1), dtype=np.uint16)
    denom = np.zeros(max(npairs, 1), dtype=np.uint16) if want_denom else None
    lib().oracle_allpairs_rows(hashes.reshape(-1), nhash, N, s, r0, r1, common,
                               denom.ctypes.data if denom is not None else None, threads)
    return common[:npairs], (denom[:npairs] if denom is not None else None)


def dist_pairs_list(hashes, nhash, s, pi, pj, threads=0):
    pi = np.ascontiguousarray(pi, dtype=np.uint32)
    pj = np.ascontiguousarray(pj, dtype=np.uint32)
    out = np.zeros(len(pi), dtype=np.uint16)
    lib().oracle_dist_pairs_list(np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1),
                                 np.ascontiguousarray(nhash, dtype=np.uint32), s, pi, pj, len(pi), out, threads)
    return out


def max_threads() -> int:
    return int(lib().oracle_max_threads())
