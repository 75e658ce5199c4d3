#!/bin/bash
# Build libdrephip.so variants for same-box A/B runs (tools/gpu_*ab.sh):
#   tools/build_ab.sh <name> [<git rev>]   -> drep_amd/lib_ab/<name>/libdrephip.so
# from the csrc of <git rev> (default: the working tree).  EXTRA passes hipcc flags.
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
name=$1; rev=$2
W=$(mktemp -d /tmp/drephip_ab.XXXXXX)
mkdir -p $W/drep_amd/csrc $W/include
if [ -n "$rev" ]; then
  git -C $ROOT archive $rev drep_amd/csrc include | tar -x -C $W
else
  cp $ROOT/drep_amd/csrc/* $W/drep_amd/csrc/; cp $ROOT/include/* $W/include/
fi
mkdir -p $ROOT/drep_amd/lib_ab/$name
make -s -j8 -C $W/drep_amd/csrc OUT=$ROOT/drep_amd/lib_ab/$name EXTRA="$EXTRA"
rm -f $ROOT/drep_amd/lib_ab/$name/*.o
rm -rf $W
echo "built drep_amd/lib_ab/$name/libdrephip.so"
