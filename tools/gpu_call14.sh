# round 4 call 14: seed spread, float64 third seed
bash tools/seed_spread.sh "gpu64:303"
