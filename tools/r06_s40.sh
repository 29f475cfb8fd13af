# round-6 session 40: split-filter launches of <= 2 splits in the XCD-grouped
# order by default -- whole GPU suite and smoke, mnist-real and gist benches,
# gist trace and PMC traffic (the order changes its fetch)
set -o pipefail
bash tools/gpu.sh tests bench:mnist-real:8 bench:gist:3 trace:gist:3 pmc:gist:3
