# F32X3 (split-bf16 fp32 contractions) + utterance-segment tiles: unit parity, conv parity, the C4 training
# tests, the C4 step clock + trace, C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/x3
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_f32x3.py -s -k "segment or conv1d_f32x3" > gpurun_out/x3/unit.log 2>&1 || { tail -30 gpurun_out/x3/unit.log; exit 1; }
tail -3 gpurun_out/x3/unit.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "conv1d_vs_torch" > gpurun_out/x3/parity.log 2>&1 || { tail -30 gpurun_out/x3/parity.log; exit 1; }
tail -2 gpurun_out/x3/parity.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_sizes.py tests/test_gpu_train.py > gpurun_out/x3/train.log 2>&1 || { tail -40 gpurun_out/x3/train.log; exit 1; }
tail -3 gpurun_out/x3/train.log
bash tools/c4_prof.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mode c2 --cpu-seconds 0 > gpurun_out/x3/c2.out 2>&1 || { tail -20 gpurun_out/x3/c2.out; exit 1; }
tail -1 gpurun_out/x3/c2.out | cut -c1-400
