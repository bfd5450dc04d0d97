#!/bin/bash
# Exact speculative segments: GPU tests for the spec path, then the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out/ex
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/ex/spec.log 2>&1 && echo SPEC_OK && \
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/ex/tests.log 2>&1 && echo TESTS_OK
rc=$?; tail -5 gpurun_out/ex/spec.log; tail -3 gpurun_out/ex/tests.log 2>/dev/null; exit $rc
