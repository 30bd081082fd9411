#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out/t
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/t/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t/pytest.log; tail -25 gpurun_out/t/pytest.log
