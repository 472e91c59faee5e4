#!/bin/bash
set -o pipefail
bash tools/r04/gpu_wave7.sh || exit 1
bash tools/r04/gpu_final_b.sh || exit 1
