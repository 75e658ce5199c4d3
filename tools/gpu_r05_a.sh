#!/bin/bash
# Round-5 first box pass: the library the tree ships vs one rebuilt on the box
# (sha256), smoke, the GPU suite without the scale tests, and the chain's
# launch counters at 10^4 (DREPHIP_DEBUG) for the host simulation of the chain.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
sha256sum drep_amd/lib/libdrephip.so > $O/lib_sha_shipped.txt
# rebuild HEAD's sources on the box into a scratch copy of the layout (the shipped library stays)
rm -rf /tmp/boxbuild && mkdir -p /tmp/boxbuild/include /tmp/boxbuild/drep_amd && cp include/drephip.h /tmp/boxbuild/include/ &&
  cp -r drep_amd/csrc /tmp/boxbuild/drep_amd/ && (cd /tmp/boxbuild/drep_amd/csrc && timeout -k 10 600 make -s -j16) > $O/boxbuild.log 2>&1 &&
  sha256sum /tmp/boxbuild/drep_amd/lib/libdrephip.so > $O/lib_sha_boxbuild.txt || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_screen.py tests/test_gpu_dist.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
DREPHIP_DEBUG=1 timeout -k 10 300 python -u tools/link_ab.py 10000 > $O/link1e4.json 2> $O/link1e4.err || { tail $O/link1e4.err; exit 1; }
grep chain $O/link1e4.err; cat $O/link1e4.json
