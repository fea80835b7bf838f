#!/bin/bash
# Full GPU pass: pytest -m gpu, then smoke(), each under its own time limit (gpurun_out/$TAG).
export TAG=${TAG:-suite} LIMIT=${LIMIT:-600} TAILN=${TAILN:-5}
export STEPS="python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu ${PYTEST_ARGS:-};python -c \"__import__('__graft_entry__').smoke()\""
bash "$(dirname "$0")/gpu_run.sh"
