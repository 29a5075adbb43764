cd /root/repo && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_own_gpu.py -k "exact_gelu" 2>&1 | tail -30
