source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 300 probe python tools/probe_rollout.py --B 4096,8192,16384 --N 200 --reps 100
run 300 probe64 python tools/probe_rollout.py --B 4096 --N 200 --dtype f64 --reps 50
run 900 gputests python -m pytest tests -m gpu -x -q
run 300 bench python bench.py
