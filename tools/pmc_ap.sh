# PMC passes over the all-pairs kernels (ap_bench.py); one pass per counter group.
# AP_N / AP_S / AP_PATH select the case; TAG names the output directories.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${AP_N:-6000}
TAG=${TAG:-ap}
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  g=$(echo $grp | cut -d' ' -f1)
  AP_ITERS=1 AP_SAMPLE=1000 AP_N=$N timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $PWD/gpurun_out/pmc${TAG}_$g -o pmc -- python tools/ap_bench.py > gpurun_out/pmc${TAG}_$g.log 2>&1 || { echo "pmc $TAG $g failed"; exit 1; }
done
