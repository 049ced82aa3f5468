#!/bin/bash
# Round-5 GPU iteration: GPU tests (stop on the first failure), then, unless the tests
# crashed / timed out (rc other than 0 or 1), the batch sweep + configs[0] bench entries.
# usage: tools/gpu_r05.sh TAG [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
SEL=${*:-tests}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
timeout -k 10 400 python -u bench.py --no-cpu --secondary "configs[0]_latency,batch_sweep" \
  > gpurun_out/${TAG}_bench.log 2>&1
rc2=$?
tail -c 300 gpurun_out/${TAG}_bench.log
exit $(( rc != 0 ? rc : rc2 ))
