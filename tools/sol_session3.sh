# speed-of-light / cache-residency probe of the two pyramid backings (round 5)
set -e
mkdir -p gpurun_out
timeout -k 10 180 tools/sol_c2 200 > gpurun_out/sol_c2_r05n.log 2>&1
echo done
