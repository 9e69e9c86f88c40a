# round 4 call 11: seed spread, float32 (three 50 000-iteration lqr_d20 runs sharing the GPU)
bash tools/seed_spread.sh "gpu32:101 gpu32:202 gpu32:303"
