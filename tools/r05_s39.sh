# PMC traffic of k_dist_split on the final source (its sha1 changed after the
# r05 profiles), then the bench lines again with the refreshed record in the
# box's profiles/pmc_traffic.json (make_profiles.py runs on the box between)
set -o pipefail
for wl in mnist-real gist; do
  bash tools/gpu.sh pmc:$wl:3 trace:$wl bench:$wl && python3 tools/make_profiles.py r05 $wl > gpurun_out/mp_$wl.log 2>&1 \
    && bash tools/gpu.sh bench:$wl:10 || exit 1
done
