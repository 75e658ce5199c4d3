#!/bin/bash
# One GPU-box call, parameterized (run from the repo root under gpurun):
#   STEPS="tests smoke bench ..." bash tools/gpu_round.sh
# Every step runs under its own time limit; the first failing step ends the
# call (no later GPU step runs after a failure).  Output under gpurun_out/$TAG.
#
# steps:
#   tests        the GPU suite in one pytest process (TESTS_K: a -k filter)
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py (configs[1], the driver's default line)
#   bench_c2     bench at configs[2] (10^4 genomes)            bench_c4  configs[4] (10^4, s = 10^4)
#   bench_dense  bench at 10^4 genomes of one species (family size 10^4: the dense all-pairs kernel)
#   bench_g2     bench --gpus 2 over gloo on the one GPU (--verify 1)
#   bench_g8     bench --gpus 8 over gloo on the one GPU (--verify 1; world-8 rehearsal)
#   dropin       tools/dropin_bench.py at DROPIN_NS (default "1000 10000"), reference leg included
#   profiles     tools/profile_round.sh (sketch) + tools/profile_allpairs.sh (CASES)
#   ab           tools/ap_ab.py: AB_VAR over AB_VALUES at AB_N genomes (AB_FAM, AB_S, AB_ROUNDS)
#   link         tools/link_ab.py at LINK_NS (chain timing, Z digest vs scipy's)
#   job          drep_amd.distributed --genomes JOB_N on JOB_W gloo ranks (JOB_ARGS)
#   rank_screen  tools/rank_screen.py (RS_ARGS)
#   scale        tools/gpu_scale.sh "$SCALE_SPECS"
#   price        tools/valu_microbench.hip (instruction prices) + the sketch hash kernel at configs[1] (tools/sketch_ablate.py)
#   dense_ab     bench at 10^4 genomes of one species once per value of DREPHIP_AP_CMASK in CMASK_VALUES (default "1 0 3 1 0 3")
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=${TAG:-round}
O=gpurun_out/$TAG
mkdir -p $O
export MASTER_ADDR=127.0.0.1

fail() { echo "step $1 failed"; [ -n "$2" ] && tail -${3:-20} "$2" | grep -v amdgpu.ids; exit 1; }
bench_line() {   # name, args...
  local n=$1; shift
  timeout -k 10 ${BENCH_LIMIT:-300} python bench.py "$@" > $O/$n.json 2> $O/$n.err || fail $n $O/$n.err
  python3 - $O/$n.json <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["kernels_rank0"]
print(sys.argv[1].split("/")[-1], "ms/step %.2f" % d["ms_per_step"], "value %.3g" % d["value"],
      "dist %.3g" % (d["dist_pairs_per_s"] or 0), "sketch %.2f ms" % k["sketch_hash_ms_avg"],
      "ap %.3f ms" % k["allpairs_ms_avg"], "screen %.3f ms" % k.get("screen_ms_avg", 0),
      "roofline.frac %.4f" % d["roofline"]["frac"], "verified", d.get("verified"), d.get("verified_against_single_gpu"))
EOF
}

for step in ${STEPS:-tests smoke bench}; do
  case $step in
    tests)
      timeout -k 10 ${TESTS_LIMIT:-1100} python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
          ${TESTS_K:+-k "$TESTS_K"} > $O/gputest.log 2>&1 || fail tests $O/gputest.log 30
      tail -2 $O/gputest.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
      tail -3 $O/smoke.log ;;
    bench) bench_line bench ;;
    bench_c2) bench_line bench_c2 --genomes 10000 --steps 3 --warmup 1 ;;
    bench_c4) bench_line bench_c4 --genomes 10000 --sketch 10000 --steps 3 --warmup 1 ;;
    bench_dense) bench_line bench_dense --genomes 10000 --family-size 10000 --steps 3 --warmup 1 ;;
    bench_g2) DREPHIP_DIST_BACKEND=gloo bench_line bench_g2 --gpus 2 --steps 3 --warmup 1 --verify 1 --cpu-baseline 0 ;;
    bench_g8) DREPHIP_DIST_BACKEND=gloo BENCH_LIMIT=400 bench_line bench_g8 --gpus 8 --steps 5 --warmup 2 --verify 1 --cpu-baseline 0 ;;
    dropin)
      for n in ${DROPIN_NS:-1000 10000}; do
        timeout -k 10 600 python tools/dropin_bench.py --genomes $n --reference-leg --out $O/dropin_$n.json \
            > $O/dropin_$n.log 2>&1 || fail dropin_$n $O/dropin_$n.log
        python3 -c "import json; d=json.load(open('$O/dropin_$n.json')); r=d.get('reference_leg',{}); print('dropin N=$n branch %.3f s (all_vs_all_MASH %.3f, cluster_mash_database %.3f); reference cluster steps %.2f s; identical' % (d['branch_s'], d['all_vs_all_MASH_s'], d['cluster_mash_database_s'], r.get('total_s', 0)), r.get('Z_identical'), r.get('linkage_db_identical'), r.get('Cdb_identical'))"
      done ;;
    profiles)
      ROUND=$TAG bash tools/profile_round.sh > $O/profile_round.log 2>&1 || fail profiles $O/profile_round.log
      ROUND=$TAG bash tools/profile_allpairs.sh > $O/profile_allpairs.log 2>&1 || fail profiles_ap $O/profile_allpairs.log
      tail -3 $O/profile_allpairs.log ;;
    ab)
      AB_VAR=$AB_VAR timeout -k 10 ${AB_LIMIT:-600} python tools/ap_ab.py ${AB_N:-10000} "$AB_VALUES" ${AB_ROUNDS:-3} \
          > $O/ab_${AB_VAR}_${AB_N:-10000}_f${AB_FAM:-100}.json 2> $O/ab.err || fail ab $O/ab.err
      grep -E "^round" $O/ab.err | tail -20 ;;
    link)
      for n in ${LINK_NS:-10000 100000}; do
        timeout -k 10 400 python tools/link_ab.py $n > $O/link_$n.json 2> $O/link_$n.err || fail link_$n $O/link_$n.err
        python3 -c "import json; d=json.load(open('$O/link_$n.json')); print('N=$n chain ms %.1f / %.1f' % (d['chain_kernel_ms_0'], d['chain_kernel_ms_1']), 'launches/merge %.4f' % d.get('launches_per_merge', 0), 'scipy digest', d['Z_equals_scipy_digest'])"
      done ;;
    job)
      DREPHIP_DIST_BACKEND=${JOB_BACKEND:-gloo} timeout -k 10 ${JOB_LIMIT:-600} python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node ${JOB_W:-1} --master-addr 127.0.0.1 --master-port 29811 -m drep_amd.distributed \
          --genomes ${JOB_N:-10000} $JOB_ARGS > $O/job.json 2> $O/job.err || fail job $O/job.err
      tail -c 1500 $O/job.json ;;
    rank_screen)
      timeout -k 10 300 python tools/rank_screen.py $RS_ARGS > $O/rank_screen.json 2> $O/rank_screen.err || fail rank_screen $O/rank_screen.err
      tail -c 1500 $O/rank_screen.json ;;
    scale) bash tools/gpu_scale.sh "$SCALE_SPECS" || exit 1 ;;
    price)
      # instruction prices at 8 waves/SIMD, then the sketch hash kernel's own time
      # at configs[1] (product library), PRICE_REPS times interleaved
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o $O/valu_microbench tools/valu_microbench.hip \
          > $O/price_build.log 2>&1 || fail price_build $O/price_build.log
      for r in $(seq ${PRICE_REPS:-2}); do
        timeout -k 10 120 $O/valu_microbench > $O/valu_microbench_$r.json 2> $O/price.err || fail price $O/price.err
        DREPHIP_SK_ONE_ROUND=1 timeout -k 10 300 python tools/sketch_ablate.py 10 > $O/sketch_ms_$r.json 2>> $O/price.err \
            || fail sketch_ms $O/price.err
        echo "rep $r: $(cat $O/sketch_ms_$r.json)"
      done
      rm -f $O/valu_microbench ;;
    dense_ab)
      for v in ${CMASK_VALUES:-1 0 3 1 0 3}; do
        DREPHIP_AP_CMASK=$v bench_line dense_cmask_$v --genomes 10000 --family-size 10000 --steps 3 --warmup 1 --cpu-baseline 0 --check 0
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
