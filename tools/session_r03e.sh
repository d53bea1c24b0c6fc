# round-3 session e: multi-rank rehearsals on the one GPU with the file rendezvous and the topology
# block (8 self-launched gloo ranks; 2 torchrun gloo ranks — the driver's launcher form, env://;
# the nccl refusal on one GPU), then config 4's in-place PMC records
exec tools/gpu_session.sh \
  "selflaunch_gloo8_c2_r03e|300|GDP_BENCH_BACKEND=gloo GDP_BENCH_RANK_LOGS=gpurun_out/ranks_gloo8 python3 bench.py --gpus 8 --steps 20 --warmup 3 --no-cpu --no-autotune" \
  "torchrun2_gloo_c2_r03e|300|GDP_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --no-autotune" \
  "selflaunch_nccl2_refused_r03e|120|python3 bench.py --gpus 2 --no-cpu; echo exit=\$?" \
  "pmc_inplace_c4_r03e|900|bash tools/pmc_inplace.sh c4 r03"
