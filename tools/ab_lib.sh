#!/bin/bash
# Same-box A/B of library builds (drep_amd/lib_ab/<name>, tools/build_ab.sh)
# against the default library on the all-pairs kernel: LIBS="default vil"
# (rounds x libraries interleaved), each run tools/ap_ab.py with the whole
# triangle checked against the literal-merge kernel, at 10^4 genomes of one
# species (family 10^4: the dense kernel), configs[2] (screened) and
# configs[1] (dense, screen off).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${TAG:-libab}
mkdir -p $O
for rd in $(seq ${ROUNDS:-2}); do
for lib in ${LIBS:-default vil}; do
  if [ $lib = default ]; then unset DREPHIP_LIB; else export DREPHIP_LIB=drep_amd/lib_ab/$lib/libdrephip.so; fi
  for cfg in "10000 10000" "10000 100"; do
    set -- $cfg
    AB_FAM=$2 AB_VAR=DREPHIP_AP_HIT timeout -k 10 300 python tools/ap_ab.py $1 1 2 > $O/$lib.$1.$2.json 2> $O/$lib.$1.$2.err || { tail -5 $O/$lib.$1.$2.err; exit 1; }
    echo "rd $rd lib $lib N $1 fam $2: $(grep -E '^round' $O/$lib.$1.$2.err | tr '\n' ' ')"
  done
  DREPHIP_AP_SCREEN=2 AB_FAM=100 AB_VAR=DREPHIP_AP_HIT timeout -k 10 300 python tools/ap_ab.py 1000 1 4 > $O/$lib.1000.json 2> $O/$lib.1000.err || exit 1
  echo "rd $rd lib $lib N 1000: $(grep -E '^round' $O/$lib.1000.err | tr '\n' ' ')"
done
done
