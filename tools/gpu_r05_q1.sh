#!/bin/bash
# Round-5 GPU suite (every gpu test, the scale tests at configs[1]-[4] and the
# dense set included), then the smoke check.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
TESTS_LIMIT=1150 bash tools/gpu_tests.sh || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/gputest.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
