# full GPU suite, default bench line, round profile set on the current tree
mkdir -p gpurun_out/r3l
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3l/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r3l/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3l/bench.json 2> gpurun_out/r3l/bench.err || exit 1
cut -c1-400 gpurun_out/r3l/bench.json
bash tools/prof_round.sh r3l_prof || exit 1
ls gpurun_out/r3l_prof gpurun_out/r3l_prof/trace gpurun_out/r3l_prof/pmc
