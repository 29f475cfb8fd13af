# round-6 session 37: gist (configs[4] shape, 500K x 960 fp32, k = 100) on
# the final build -- bench, steady trace, PMC traffic passes (its
# pmc_traffic.json entry was measured on round 5's k_dist_split)
set -o pipefail
bash tools/gpu.sh bench:gist:3 trace:gist:3 pmc:gist:3
