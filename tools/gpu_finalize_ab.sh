#!/bin/bash
# GPU-box A/B of the sketch finalize kernels (bucket sort vs bitonic) after the
# parity tests: configs[1] bench and an s = 10^4 bench, per-kernel averages.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for f in 1 0; do
  DREPHIP_FINALIZE=$f timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/fin$f.json 2>/dev/null || exit 1
  DREPHIP_FINALIZE=$f timeout -k 10 300 python bench.py --cpu-baseline 0 --genomes 2000 --sketch 10000 --steps 3 --warmup 1 > gpurun_out/fin${f}_s1e4.json 2>/dev/null || exit 1
done
python - <<'P'
import json
for f in ("fin1", "fin0", "fin1_s1e4", "fin0_s1e4"):
    d = json.load(open("gpurun_out/%s.json" % f)); k = d["kernels_rank0"]
    print(f, round(d["ms_per_step"], 3), {a: round(b, 4) for a, b in k.items() if a.endswith("avg")})
P
