#!/bin/bash
# The GPU test suite on the box (run from the repo root), one pytest process,
# every test under its own thread timeout; log in gpurun_out/gputest.log.
# Extra pytest arguments (e.g. -k) pass through.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 ${TESTS_LIMIT:-1100} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 900 --timeout-method thread "$@" \
    > gpurun_out/gputest.log 2>&1
rc=$?
tail -5 gpurun_out/gputest.log
exit $rc
