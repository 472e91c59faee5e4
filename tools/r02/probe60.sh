#!/usr/bin/env bash
# Round-2 probe 60 (change reverted after it segfaulted): RCCL send/recv captured into the exchange-mode step graph
# (peer == self on one GPU), then the halo / multiproc suites.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe60
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_halo.py -k "captured" -x -v --timeout 120 --timeout-method thread > "$O/captured.log" 2>&1
tail -n 8 "$O/captured.log"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_halo.py tests/test_gpu_multiproc.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
