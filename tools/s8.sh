source tools/gpu_steps.sh
run 300 probe python tools/probe_rollout.py --B 2048,4096,8192,16384,32768 --N 200 --reps 100
run 300 probe_n python tools/probe_rollout.py --B 4096 --N 200 --reps 100 --scheme naive
run 900 pytest_gpu python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider
run 300 bench python bench.py --steps 200 --warmup 20 --no-cpu-baseline
