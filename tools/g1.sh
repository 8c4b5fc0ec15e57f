set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_parity_gpu.py -k "both_kernels" > gpurun_out/t2_tests.log 2>&1
timeout -k 10 300 python -u tools/kbench.py --series 2000 --cases tile:linear:60,tile2:linear:60,tile:linear:60,tile2:linear:60,tile2:linear:20,tile:linear:20 > gpurun_out/t2_kb.jsonl 2>&1
