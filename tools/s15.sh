source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 200 diag_new python tools/diag_fp32.py VDP 20 naive cost
run 900 gputests python -m pytest tests -m gpu -x -q
run 300 probe python tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
run 300 probe_vdp python tools/probe_rollout.py --B 4096 --N 200 --eqn VDP --reps 20
