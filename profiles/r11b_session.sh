timeout -k 10 300 python -u -m pytest tests/test_gpu_labels.py -x -v --timeout 120 --timeout-method thread -k mutations > gpurun_out/r11b.log 2>&1; tail -40 gpurun_out/r11b.log
