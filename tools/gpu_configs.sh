# BASELINE.json configs[2] and configs[4] at 1 GPU (development measurement)
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --genomes 10000 --sketch 1000 --steps 3 --warmup 1 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "c2 failed"; tail gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 300 python bench.py --genomes 10000 --sketch 10000 --steps 2 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "c4 failed"; tail gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
