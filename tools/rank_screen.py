"""The all-pairs stage of one rank of a W-way sharded job, timed on one GPU (not
product code): synthetic families (the bench generator) sketched on the device,
then drephip_allpairs_device over each rank's row range (parallel.row_partition),
the screen forced on, HIP-event times of the screen and of the LIST kernel per
range, against the whole triangle.  RS_N genomes of RS_L bp, sketch RS_S, RS_W ranks.
With the sharded screen (RS_SHARD=1, the default): each rank's hash part
(drephip_screen_part) timed, then each rank's rows screened from the cell words
and records routed to it (drephip_allpairs_device_marked: cells OR-ed in, pair
map, lists) and its LIST kernel, the rank's segment compared with the
unsharded call's.  The exchange itself (one all-to-all of 16-byte records) is
sized, not timed: one GPU holds every part here.
usage: RS_N=10000 RS_S=10000 RS_W=8 python tools/rank_screen.py"""
import json
import os
import sys

import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from drep_amd import _lib, parallel

N = int(os.environ.get("RS_N", 10000)); L = int(os.environ.get("RS_L", 5_000_000))
s = int(os.environ.get("RS_S", 10000)); W = int(os.environ.get("RS_W", 8))
ctx = _lib.Context(0, 21, s, 42)
ctx.set_timing(True)
ctx.set_allpairs_screen(ctx.SCREEN_ON)
ST = torch.cuda.current_stream().cuda_stream
tile = _lib.tile_bases(); P = _lib.padded_bases([L]); tot = tile + N * P
codes = torch.zeros(tot // 16, dtype=torch.int32, device="cuda")
valid = torch.zeros(tot // 32, dtype=torch.int32, device="cuda")
ctx.synth_device(0xD2E9, 0, N, 100, L, codes.data_ptr(), valid.data_ptr(), ST)
h = torch.full((N, s), -1, dtype=torch.int64, device="cuda"); n = torch.zeros(N, dtype=torch.int32, device="cuda")
off = np.array([tile + i * P for i in range(N)], np.uint64)
ctx.sketch_device(codes.data_ptr(), valid.data_ptr(), off, np.full(N, P, np.uint64), np.full(N, L - 20, np.uint64), N,
                  h.data_ptr(), n.data_ptr(), ST)
del codes, valid
bounds = parallel.row_partition(N, W)
res = {"N": N, "s": s, "L": L, "W": W, "build_id": _lib.build_id(), "ranges": []}


def timed(r0, r1, reps=3):
    npairs = parallel.cond_start(r1, N) - parallel.cond_start(r0, N)
    out = torch.zeros(max(npairs, 1), dtype=torch.int16, device="cuda")
    best = None
    for _ in range(reps + 1):
        ctx.allpairs_device(h.data_ptr(), n.data_ptr(), N, r0, r1, out.data_ptr(), None, ST)
        torch.cuda.synchronize()
        t = (ctx.kernel_ms(4)[0], ctx.kernel_ms(2)[0])
        best = t if best is None or sum(t) < sum(best) else best
    st = ctx.screen_stats()
    return {"rows": [r0, r1], "pairs": npairs, "screen_ms": best[0], "list_kernel_ms": best[1],
            "marked": st["marked"], "written_by_screen": st["simple"]}


res["whole"] = timed(0, N)
for r0, r1 in bounds:
    res["ranges"].append(timed(r0, r1))

if os.environ.get("RS_SHARD", "1") != "0":
    R = ctx.screen_geometry()
    cells, recs, parts, checks = [], [], [], 0
    for p in range(W):
        best = None
        for _ in range(4):
            c, ncell, nrec = ctx.screen_part(h.data_ptr(), n.data_ptr(), N, p, W, ST)
            t = ctx.kernel_ms(4)[0]
            best = t if best is None or t < best else best
        cl = torch.empty((max(ncell, 1), 4), dtype=torch.int32, device="cuda")
        rec = torch.empty((max(nrec, 1), 4), dtype=torch.int32, device="cuda")
        ctx.screen_part_copy(cl.data_ptr(), rec.data_ptr(), ST)
        cells.append(cl[:ncell])
        recs.append(rec[:nrec])
        checks += c
        parts.append({"part": p, "screen_part_ms": best, "cells": ncell, "records": nrec, "checks": c,
                      "bytes_sent": 16 * (ncell + nrec)})
    cells = torch.cat(cells).contiguous()
    recs = torch.cat(recs).contiguous()
    shard = {"rows_per_tile": R, "cells": int(len(cells)), "records": int(len(recs)), "checks": checks,
             "screen_used": ctx.screen_worth(N, checks)[1], "parts": parts, "ranges": []}
    for p, (r0, r1) in enumerate(bounds):
        npairs = parallel.cond_start(r1, N) - parallel.cond_start(r0, N)
        out = torch.zeros(max(npairs, 1), dtype=torch.int16, device="cuda")
        # what this rank receives (the job routes each cell / record to its row's owner)
        mc = cells[(cells[:, 0].to(torch.int64) * R >= r0) & (cells[:, 0].to(torch.int64) * R < r1)].contiguous()
        mr = recs[(recs[:, 0] >= r0) & (recs[:, 0] < r1)].contiguous()
        best = None
        for _ in range(4):
            ctx.allpairs_device_marked(h.data_ptr(), n.data_ptr(), N, r0, r1, out.data_ptr(), None,
                                       mc.data_ptr() if len(mc) else None, len(mc),
                                       mr.data_ptr() if len(mr) else None, len(mr), ST)
            torch.cuda.synchronize()
            t = (ctx.kernel_ms(4)[0], ctx.kernel_ms(2)[0])
            best = t if best is None or sum(t) < sum(best) else best
        st = ctx.screen_stats()
        ref = torch.zeros(max(npairs, 1), dtype=torch.int16, device="cuda")
        ctx.allpairs_device(h.data_ptr(), n.data_ptr(), N, r0, r1, ref.data_ptr(), None, ST)
        torch.cuda.synchronize()
        shard["ranges"].append({"rows": [r0, r1], "pairs": npairs, "screen_part_ms": parts[p]["screen_part_ms"],
                                "screen_finish_ms": best[0], "list_kernel_ms": best[1],
                                "screen_ms": parts[p]["screen_part_ms"] + best[0],
                                "cells_received": int(len(mc)), "records_received": int(len(mr)),
                                "bytes_received": 16 * int(len(mc) + len(mr)),
                                "marked": st["marked"], "written_by_screen": st["simple"],
                                "equal_to_unsharded": bool(torch.equal(out[:npairs], ref[:npairs]))})
    res["sharded"] = shard
print(json.dumps(res))
