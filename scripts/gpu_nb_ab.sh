set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD:$PWD/tests/golden
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_next.py -k "nibble or variants or reconstruct_crc_batch" > gpurun_out/nb_tests.log 2>&1 && \
timeout -k 10 120 python -u scripts/ab.py c3r crc_variant 0,61,62,65,66,67 5 > gpurun_out/nb_ab_c3r.log 2>&1 && \
timeout -k 10 120 python -u scripts/ab.py c5dev crc_variant 0,61,62,63,64,65,67 5 > gpurun_out/nb_ab_c5dev.log 2>&1
rc=$?; tail -3 gpurun_out/nb_tests.log; cat gpurun_out/nb_ab_c3r.log gpurun_out/nb_ab_c5dev.log; exit $rc
