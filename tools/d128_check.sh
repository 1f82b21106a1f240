set -e
timeout -k 10 300 python -u -m pytest tests/test_flash_attn.py -m gpu -x -q --timeout 120 --timeout-method thread -k "128 and False and 0.0" > gpurun_out/d128_tests.txt 2>&1
for r in 1 2; do for c in D128 D128b16; do for i in auto hip; do
  timeout -k 10 120 python tools/tiles_r03.py --cfg $c --mode fwd --launches 100 --impl $i >> gpurun_out/d128_time.txt 2>&1
done; done; done
