#!/bin/bash
# Round 5 s30: the seam's cross-stream ordering under device-side delays (tests/test_gpu_stream_delay.py:
# a ~200-us sleeping wave in front of every batch copy and key append on its stream).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_stream_delay.py tests/test_gpu_jitter.py > gpurun_out/s30_delay.log 2>&1
echo "rc=$?"
