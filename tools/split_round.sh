set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad_k1.py tests/test_gpu_parity.py -k "split or conv1d_vs_torch or k1" > gpurun_out/ab/split.log 2>&1 || { tail -30 gpurun_out/ab/split.log; exit 1; }
tail -2 gpurun_out/ab/split.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_sizes.py tests/test_gpu_train.py tests/test_gpu_fullsize.py > gpurun_out/ab/split_train.log 2>&1 || { tail -30 gpurun_out/ab/split_train.log; exit 1; }
tail -2 gpurun_out/ab/split_train.log
bash tools/train_tune_ab.sh "" "splitk_cfg=3"
