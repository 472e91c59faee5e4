#!/bin/bash
# Round 6, call X: fresh SQ counters of the final tree's production launches
# (headline loop, 8-way band, 32768^2 grey) — the round-5 script, output in
# gpurun_out/r06/pmc (two passes per loop, each its own rocprofv3 run).
set -o pipefail
O=gpurun_out/r06/pmc bash tools/r05/gpu_pmc.sh
