set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_model.py -m gpu -q -x -p no:cacheprovider > gpurun_out/t_model.log 2>&1; rc=$?; tail -5 gpurun_out/t_model.log; exit $rc
