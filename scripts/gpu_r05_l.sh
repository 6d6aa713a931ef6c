#!/bin/bash
# full GPU suite after the A/B split (product: version 5 at d = 768; version 6 and the retired sweeps in the A/B
# library's checks), then the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05l
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05l/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r05l/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r05l/bench.json 2> gpurun_out/r05l/bench.err && cat gpurun_out/r05l/bench.json
