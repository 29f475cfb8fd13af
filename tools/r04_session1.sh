# round-4 measurement session 1: tests, mnist + sift bench / trace / PMC
set -o pipefail
bash tools/gpu.sh tests bench:mnist:20 trace:mnist pmc:mnist:1 bench:sift:3 trace:sift:3 pmc:sift:1
