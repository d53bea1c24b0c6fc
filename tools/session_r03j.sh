# round-3 session j: final-tree evidence — GPU suite, smoke, host ASan/UBSan driver, the driver's
# default command under rocprofv3 --kernel-trace --stats, PMC records of every config-2 build
# instance (each counter its own pass), and the bench lines of configs 4 / 5 and the other ops
exec tools/gpu_session.sh \
  "gputest_r03j|600|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "smoke_r03j|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "asan_r03j|300|make -s -C tools/asan run" \
  "prof_default_r03j|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default_r03j -o run --output-format csv -- python3 bench.py" \
  "pmcv_fetch_c2_r03j|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcv_fetch_c2 -o run --output-format csv -- python3 tools/pmc_variants.py --config c2 --manifest gpurun_out/pmcv_manifest_c2.json" \
  "pmcv_write_c2_r03j|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcv_write_c2 -o run --output-format csv -- python3 tools/pmc_variants.py --config c2 --manifest gpurun_out/pmcv_manifest_c2.json"
