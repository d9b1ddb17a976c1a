#!/bin/bash
# Whole GPU suite (one process), then smoke(); output under gpurun_out/.
set -o pipefail
O=gpurun_out/${1:-suite}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu \
  > ${O}_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1
