#!/bin/bash
# GPU parity tests only: tools/gpu_pytest.sh [pytest -k expr]
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 120 --timeout-method thread ${1:+-k "$1"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -15; exit $rc
