"""Mash ``.msh`` sketch files (Cap'n Proto messages): reader and writer.

The reference keeps one ``.msh`` per genome under
``MASH_files/sketches/chunk_<i>/`` and pastes them into ``chunk_all.msh`` and
``ALL.msh`` (drep/d_cluster.py:531-567).  This module lets the MI355X path read
those files (sketch cache across runs; the reference's fixture sketches) and
write the same layout back.

Layout (decoded from the reference fixtures
tests/test_solutions/ecoli_wd/data/MASH_files/; Mash's .capnp schema is not in
the reference, so field names beyond these are inferred -- SURVEY.md 8(c)):

* root struct ``MinHash``: data words = 3; u32 @byte0 kmerSize, u32 @byte8
  sketch size (minHashesPerWindow), bool bit 96 ``concatenated`` (1), u32
  @byte20 = hashSeed XOR 42 (Cap'n Proto default-XOR; 0 for seed 42).
  Pointers: [0] -> struct{ptr[0] -> List(Reference)} (the reference list),
  [1] -> struct{ptr[0] -> empty list} (locus list).
* ``Reference`` (composite list element, 2 data words, 6 pointers):
  u64 @byte8 = length; ptr[2] name (Text), ptr[3] comment (Text),
  ptr[5] hashes64 (List(UInt64), ascending).

Only plain pointers, far pointers (single and double) and the list kinds the
format uses are implemented.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np

__all__ = ["MashReference", "MashSketchFile", "read_msh", "write_msh"]


@dataclass
class MashReference:
    name: str
    comment: str
    length: int
    hashes: np.ndarray  # uint64, ascending


@dataclass
class MashSketchFile:
    kmer: int
    sketch_size: int
    seed: int
    references: List[MashReference] = field(default_factory=list)


class _Msg:
    def __init__(self, buf: bytes):
        nseg = struct.unpack_from("<I", buf, 0)[0] + 1
        sizes = struct.unpack_from("<%dI" % nseg, buf, 4)
        off = 4 + 4 * nseg
        off += (-off) % 8
        self.segs = []
        for sz in sizes:
            self.segs.append(np.frombuffer(buf, dtype="<u8", count=sz, offset=off))
            off += 8 * sz
        self.buf = buf
        self.seg_off = []
        off = 4 + 4 * nseg
        off += (-off) % 8
        for sz in sizes:
            self.seg_off.append(off)
            off += 8 * sz

    def word(self, seg: int, idx: int) -> int:
        return int(self.segs[seg][idx])

    def resolve(self, seg: int, idx: int):
        """Follow a pointer at (seg, idx); return (seg, target_word, ptr_word)."""
        p = self.word(seg, idx)
        kind = p & 3
        if kind == 2:  # far pointer
            double = (p >> 2) & 1
            land = (p >> 3) & 0x1FFFFFFF
            tseg = p >> 32
            if not double:
                return self.resolve(tseg, land)
            # double-far: landing pad = far ptr to content + tag word
            far2 = self.word(tseg, land)
            tag = self.word(tseg, land + 1)
            cseg = far2 >> 32
            cword = (far2 >> 3) & 0x1FFFFFFF
            return cseg, cword, tag
        off = (p >> 2) & 0x3FFFFFFF
        if off & 0x20000000:
            off -= 0x40000000
        return seg, idx + 1 + off, p

    def struct_at(self, seg: int, idx: int):
        tseg, tw, p = self.resolve(seg, idx)
        if p == 0:
            return None
        assert p & 3 == 0, "expected struct pointer"
        dw = (p >> 32) & 0xFFFF
        pc = (p >> 48) & 0xFFFF
        return (tseg, tw, dw, pc)

    def list_at(self, seg: int, idx: int):
        tseg, tw, p = self.resolve(seg, idx)
        if p == 0:
            return None
        assert p & 3 == 1, "expected list pointer"
        esz = (p >> 32) & 7
        cnt = p >> 35
        return (tseg, tw, esz, cnt)

    def text_at(self, seg: int, idx: int) -> str:
        lst = self.list_at(seg, idx)
        if lst is None:
            return ""
        tseg, tw, esz, cnt = lst
        assert esz == 2
        start = self.seg_off[tseg] + 8 * tw
        raw = self.buf[start:start + cnt]
        return raw.rstrip(b"\x00").decode("utf-8", "replace")


def read_msh(path_or_bytes) -> MashSketchFile:
    """Read a Mash ``.msh`` (Cap'n Proto) sketch file."""
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
        buf = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as fh:
            buf = fh.read()
    m = _Msg(buf)
    root = m.struct_at(0, 0)
    rseg, rw, rdw, rpc = root
    d0 = m.word(rseg, rw) if rdw > 0 else 0
    d1 = m.word(rseg, rw + 1) if rdw > 1 else 0
    d2 = m.word(rseg, rw + 2) if rdw > 2 else 0
    kmer = d0 & 0xFFFFFFFF
    ssize = d1 & 0xFFFFFFFF
    seed = ((d2 >> 32) & 0xFFFFFFFF) ^ 42
    out = MashSketchFile(kmer=kmer, sketch_size=ssize, seed=seed)
    rl = m.struct_at(rseg, rw + rdw + 0)
    if rl is None:
        return out
    lseg, lw, ldw, lpc = rl
    lst = m.list_at(lseg, lw + ldw)
    if lst is None:
        return out
    eseg, ew, esz, wcount = lst
    assert esz == 7, "references must be a composite list"
    tag = m.word(eseg, ew)
    n = (tag >> 2) & 0x3FFFFFFF
    edw = (tag >> 32) & 0xFFFF
    epc = (tag >> 48) & 0xFFFF
    stride = edw + epc
    for i in range(n):
        base = ew + 1 + i * stride
        length = m.word(eseg, base + 1) if edw > 1 else 0
        pbase = base + edw
        name = m.text_at(eseg, pbase + 2) if epc > 2 else ""
        comment = m.text_at(eseg, pbase + 3) if epc > 3 else ""
        hashes = np.zeros(0, dtype=np.uint64)
        if epc > 5:
            hl = m.list_at(eseg, pbase + 5)
            if hl is not None:
                hseg, hw, hsz, hcnt = hl
                assert hsz == 5, "hashes64 must be a List(UInt64)"
                hashes = np.array(m.segs[hseg][hw:hw + hcnt], dtype=np.uint64)
        out.references.append(MashReference(name, comment, int(length), hashes))
    return out


# ------------------------------------------------------------------ writer
def _struct_ptr(off: int, dw: int, pc: int) -> int:
    return ((off & 0x3FFFFFFF) << 2) | (dw << 32) | (pc << 48)


def _list_ptr(off: int, esz: int, cnt: int) -> int:
    return 1 | ((off & 0x3FFFFFFF) << 2) | (esz << 32) | (cnt << 35)


def _text_words(text: str) -> np.ndarray:
    """A Cap'n Proto Text blob: UTF-8 bytes + NUL, zero-padded to whole words."""
    raw = text.encode("utf-8") + b"\x00"
    nw = (len(raw) + 7) // 8
    return np.frombuffer(raw + b"\x00" * (8 * nw - len(raw)), dtype="<u8"), len(raw)


def write_msh(path: str, refs: Sequence[MashReference], kmer: int = 21,
              sketch_size: int = 1000, seed: int = 42) -> None:
    """Write ``refs`` as a single-segment Cap'n Proto ``.msh`` message with the
    structure :func:`read_msh` reads (the layout of the reference fixtures).
    The message is sized up front and filled in one uint64 array (hash lists
    are slice copies), in this word order: root pointer, root struct, the
    reference-list holder, the locus holder and its empty list tag, the
    references' composite list, then per reference its name, comment and hash
    list."""
    n = len(refs)
    edw, epc = 2, 6
    texts = [(_text_words(r.name), _text_words(r.comment)) for r in refs]
    hashes = [np.asarray(r.hashes, dtype=np.uint64) for r in refs]
    tag = 9
    total = tag + 1 + n * (edw + epc) + sum(len(a[0]) + len(b[0]) + len(h) for (a, b), h in zip(texts, hashes))
    w = np.zeros(total, dtype="<u8")
    root_ptr, root, holder, locus, ltag = 0, 1, 6, 7, 8
    w[root_ptr] = _struct_ptr(root - root_ptr - 1, 3, 2)
    w[root + 0] = kmer & 0xFFFFFFFF
    w[root + 1] = (sketch_size & 0xFFFFFFFF) | (1 << 32)   # concatenated = true
    w[root + 2] = ((seed ^ 42) & 0xFFFFFFFF) << 32
    w[root + 3] = _struct_ptr(holder - (root + 3) - 1, 0, 1)
    w[root + 4] = _struct_ptr(locus - (root + 4) - 1, 0, 1)
    # locus list: empty list of structs (tag-only composite list)
    w[locus] = _list_ptr(ltag - locus - 1, 7, 0)
    # references composite list
    w[holder] = _list_ptr(tag - holder - 1, 7, n * (edw + epc))
    w[tag] = (n << 2) | (edw << 32) | (epc << 48)
    at = tag + 1 + n * (edw + epc)
    for i, (r, (name, comment), h) in enumerate(zip(refs, texts, hashes)):
        base = tag + 1 + i * (edw + epc)
        w[base + 1] = int(r.length) & 0xFFFFFFFFFFFFFFFF
        pbase = base + edw
        for slot, (tw, nbytes) in ((2, name), (3, comment)):
            w[at:at + len(tw)] = tw
            w[pbase + slot] = _list_ptr(at - (pbase + slot) - 1, 2, nbytes)
            at += len(tw)
        w[pbase + 5] = _list_ptr(at - (pbase + 5) - 1, 5, len(h))
        w[at:at + len(h)] = h
        at += len(h)
    header = struct.pack("<II", 0, total)
    tmp = path + ".tmp%d" % os.getpid()
    with open(tmp, "wb") as fh:
        fh.write(header)
        fh.write(w.tobytes())
    os.replace(tmp, path)
