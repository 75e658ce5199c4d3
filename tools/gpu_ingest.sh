#!/bin/bash
# FASTA ingest measurement on the GPU box (tools/ingest_bench.py), printed short.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ingest_bench.py ${COPIES:-250} > gpurun_out/ingest.json 2> gpurun_out/ingest.err || { tail -5 gpurun_out/ingest.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/ingest.json"))
for k in ("plain_first_call", "plain", "gzip"):
    print(k, {x: round(d[k][x], 4) for x in ("wall_s", "Mbp_per_s", "library_wall_s", "host_read_pack_s", "read_parse_thread_s", "pack_thread_s", "device_s", "batches")})
print(d["dropin_all_vs_all_MASH"])
PY
