# Fuse-depth sweep (auto shape) on the large BASELINE frames and the headline frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/band_sweep.py --worlds 1 --fuse 2,3,4,5,6,8,10,12,16 --channels grey --width 32768 --height 32768 --iters 2 --shapes auto > gpurun_out/fuse_32768grey.txt 2>&1 &&
timeout -k 10 200 python -u tools/band_sweep.py --worlds 1,8 --fuse 2,3,4,5,6,8,10,12,16 --width 8192 --height 8192 --iters 4 --shapes auto > gpurun_out/fuse_8192rgb.txt 2>&1 &&
timeout -k 10 200 python -u tools/band_sweep.py --worlds 1,8 --fuse 2,3,4,5,6,8,10,12,16 --width 32768 --height 32768 --channels grey --iters 2 --shapes auto > gpurun_out/fuse_32768grey_w8.txt 2>&1 &&
timeout -k 10 200 python -u tools/band_sweep.py --worlds 1,2,4,8 --fuse 4,5,6,8,10,12,16 --iters 10 --shapes auto > gpurun_out/fuse_1920rgb.txt 2>&1
