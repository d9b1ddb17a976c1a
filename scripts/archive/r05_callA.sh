#!/bin/bash
# round 5 call A: the doorbell shutdown contract tests, then the exit-order probe
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_evp_shutdown.py tests/test_evp_doorbell.py tests/test_evp_multi_device.py > $O/tests.log 2>&1 || exit $?
cd tools
timeout -k 10 60 ./exit_order_probe nohip > ../$O/probe_nohip.txt 2>&1; echo "rc=$?" >> ../$O/probe_nohip.txt
timeout -k 10 60 ./exit_order_probe hip > ../$O/probe_hip.txt 2>&1; echo "rc=$?" >> ../$O/probe_hip.txt
