#!/bin/bash
# Which resource binds k_sketch_hash21: same-box hash-kernel timing at
# configs[1] (tools/sketch_ablate.py), product library vs the ablation build
# (lib_ab/skabl: table indices ANDed with DREPHIP_SK_KMASK) with real indices
# (0x3FF: +5 VALU per k-mer) and with every lane reading entry 0 (0: LDS
# broadcast, no bank conflicts, the same instructions), and the no-LDS build
# (lib_ab/sknolds: table entries taken from the k-mer's own words, 58.1
# instead of 63.1 VALU per k-mer, no LDS read), interleaved.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r05skabl
mkdir -p $O
for rep in 1 2; do
  for V in product real bcast nolds; do
    case $V in
      product) unset DREPHIP_LIB DREPHIP_SK_KMASK ;;
      real) export DREPHIP_LIB=drep_amd/lib_ab/skabl/libdrephip.so DREPHIP_SK_KMASK=0x3FF ;;
      bcast) export DREPHIP_LIB=drep_amd/lib_ab/skabl/libdrephip.so DREPHIP_SK_KMASK=0 ;;
      nolds) export DREPHIP_LIB=drep_amd/lib_ab/sknolds/libdrephip.so; unset DREPHIP_SK_KMASK ;;
    esac
    DREPHIP_SK_ONE_ROUND=1 timeout -k 10 200 python tools/sketch_ablate.py 10 > $O/$V.$rep.json 2> $O/$V.$rep.err \
        || { echo "$V failed"; tail -5 $O/$V.$rep.err; exit 1; }
    echo "$V rep $rep: $(cat $O/$V.$rep.json)" | tee -a $O/summary.txt
  done
done
unset DREPHIP_LIB DREPHIP_SK_KMASK
