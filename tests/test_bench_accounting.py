"""bench.py's roofline accounting, pinned to SURVEY.md §8(d)'s table of algorithmic bytes
(B = 4·H·W + 4·(S+3)·P per image, P = Σ_o H_o·W_o) and its per-config pyramid sizes."""
import os
import re
import sys

import pytest
from conftest import BUILD_VARIANTS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


@pytest.mark.parametrize("H,W,O,P,B", [
    (512, 512, 4, 348_160, 8_011_776),             # config 1
    (4096, 4096, 5, 22_347_776, 514_064_384),      # config 2 (and 4, per image)
    (1080, 1920, 5, 2_762_040, 63_535_200),        # config 3, per image
    (16384, 16384, 5, 357_564_416, 8_225_030_144),  # config 5
])
def test_algorithmic_bytes_match_survey_table(H, W, O, P, B):
    assert bench.pyramid_pixels(H, W, O) == P
    assert bench.algorithmic_bytes(H, W, 2, O, 1) == B


def test_batch_and_uint8_accounting():
    one = bench.algorithmic_bytes(1080, 1920, 2, 5, 1)
    assert bench.algorithmic_bytes(1080, 1920, 2, 5, 64) == 64 * one == 4_066_252_800
    # uint8 input: a quarter of the input bytes, the same pyramid bytes
    assert bench.algorithmic_bytes(4096, 4096, 2, 5, 1, in_bytes=1) == 514_064_384 - 3 * 4096 * 4096


def test_configs_are_the_baseline_workloads():
    c = bench.CONFIGS
    assert (c["c2"]["H"], c["c2"]["W"], c["c2"]["batch"], c["c2"]["O"]) == (4096, 4096, 1, 5)
    assert (c["c3"]["H"], c["c3"]["W"], c["c3"]["batch"]) == (1080, 1920, 64)
    assert (c["c4"]["H"], c["c4"]["batch"]) == (4096, 64)
    assert c["c5"]["H"] == 16384 and c["c5"]["band"]


def test_rotation_exceeds_the_infinity_cache():
    # config 2's per-step working set (514 MB) is rotated over enough sets to exceed 2 GiB (8x MALL)
    set_bytes = bench.algorithmic_bytes(4096, 4096, 2, 5, 1)
    rotate = max(1, -(-bench.ROTATE_BYTES // set_bytes))
    assert rotate == 5 and rotate * set_bytes >= 8 * (256 << 20)


_RANK_PROBE = r"""
import json, os, sys, time
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GDP_BENCH_RDV")
with open(os.path.join(sys.argv[1], "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({"env": {k: os.environ.get(k) for k in keys}, "argv": sys.argv[1:]}, f)
if len(sys.argv) > 2 and sys.argv[2] == "fail-rank1":
    if os.environ["RANK"] == "1":
        sys.stderr.write("rank 1 failing on purpose\n")
        sys.exit(3)
    time.sleep(600)  # a rank left waiting in a collective: the launcher must stop it
"""


def test_bench_launches_its_own_ranks(tmp_path, monkeypatch, capfd):
    """`bench.py --gpus N` with no launcher starts N ranks itself: each child
    gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1, NO MASTER_PORT (VERDICT r2 item 2:
    the ranks meet through a file rendezvous in a fresh private directory, GDP_BENCH_RDV, so no
    port can be taken between its choice and its bind) and the parent's arguments; a failing
    rank's status is returned, its stderr kept under GDP_BENCH_RANK_LOGS and its tail printed,
    and the other ranks are stopped."""
    import json
    import time

    import bench

    probe = tmp_path / "probe.py"
    probe.write_text(_RANK_PROBE)
    logs = tmp_path / "logs"
    monkeypatch.setenv("GDP_BENCH_RANK_LOGS", str(logs))
    monkeypatch.setenv("MASTER_PORT", "29500")  # a stale port in the parent's env is not inherited
    assert bench.launch_ranks(3, [str(tmp_path), "ok"], script=str(probe)) == 0
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    rdv = {r["env"]["GDP_BENCH_RDV"] for r in recs}
    assert len(rdv) == 1
    rdv = rdv.pop()
    assert rdv and not os.path.exists(os.path.dirname(rdv))  # private directory, removed afterwards
    for r, rec in enumerate(recs):
        assert rec["env"]["RANK"] == rec["env"]["LOCAL_RANK"] == str(r)
        assert rec["env"]["WORLD_SIZE"] == rec["env"]["LOCAL_WORLD_SIZE"] == "3"
        assert rec["env"]["MASTER_ADDR"] == "127.0.0.1"
        assert rec["env"]["MASTER_PORT"] is None
        assert rec["argv"] == [str(tmp_path), "ok"]
    t0 = time.time()
    capfd.readouterr()
    assert bench.launch_ranks(2, [str(tmp_path), "fail-rank1"], script=str(probe)) == 3
    assert time.time() - t0 < 60  # rank 0 (sleeping) was stopped, not waited for
    assert "rank 1 failing on purpose" in (logs / "rank1.stderr").read_text()
    err = capfd.readouterr().err
    assert "rank 1 exited with 3" in err and "rank 1 failing on purpose" in err and str(logs / "rank1.stderr") in err
    # without GDP_BENCH_RANK_LOGS the failing rank's log survives in a private directory it names
    monkeypatch.delenv("GDP_BENCH_RANK_LOGS")
    assert bench.launch_ranks(2, [str(tmp_path), "fail-rank1"], script=str(probe)) == 3
    err = capfd.readouterr().err
    path = err.split("Its stderr (", 1)[1].split(")", 1)[0]
    assert os.path.exists(path) and "failing on purpose" in open(path).read()
    import shutil

    shutil.rmtree(os.path.dirname(path))


def test_launcher_stopped_by_a_signal_stops_its_ranks(tmp_path):
    """A launcher that is itself told to stop (SIGTERM from a timeout) stops its ranks instead of
    leaving them running on the GPUs."""
    import signal
    import subprocess
    import time

    sleeper = tmp_path / "sleeper.py"
    sleeper.write_text("import os, sys, time\nopen(os.path.join(sys.argv[1], 'pid%s' % os.environ['RANK']), 'w')"
                       ".write(str(os.getpid()))\ntime.sleep(600)\n")
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, [%r], script=%r))" % (REPO, str(tmp_path), str(sleeper)))
    parent = subprocess.Popen([sys.executable, "-c", code])
    for _ in range(400):
        if all((tmp_path / f"pid{r}").exists() and (tmp_path / f"pid{r}").read_text() for r in range(2)):
            break
        time.sleep(0.05)
    pids = [int((tmp_path / f"pid{r}").read_text()) for r in range(2)]
    parent.send_signal(signal.SIGTERM)
    assert parent.wait(timeout=60) != 0

    def running(pid):  # gone, or a zombie waiting to be reaped
        try:
            with open(f"/proc/{pid}/status") as f:
                return not any(line.startswith("State:") and "Z" in line for line in f)
        except OSError:
            return False

    deadline = time.time() + 10
    while any(running(p) for p in pids) and time.time() < deadline:
        time.sleep(0.1)
    assert not any(running(p) for p in pids), pids


def test_rank_topology_assembly(monkeypatch):
    """The N-rank line certifies itself: rank_topology gathers every rank's
    device identity and counts the ranks with an all_reduce of ones.  A gloo rehearsal with two
    ranks on one device says so explicitly; under nccl the same shared device is fatal."""
    import types

    import bench

    class FakeDist:
        def __init__(self, devs, count):
            self.devs, self.count = devs, count

        def all_gather_object(self, out, obj):
            out[:] = self.devs

        def all_reduce(self, t):
            t.fill_(self.count)

    props = types.SimpleNamespace(name="AMD Instinct MI355X", pci_domain_id=0, pci_bus_id=0x75, pci_device_id=0,
                                  uuid="GPU-aa")
    import torch

    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props)
    args = types.SimpleNamespace(gpus=2)
    same = [{"rank": r, "device": 0, "pci": "0000:75:00.0", "uuid": "GPU-aa"} for r in range(2)]
    topo = bench.rank_topology(2, 0, 0, "gloo", FakeDist(same, 2), args)
    assert topo["backend"] == "gloo" and topo["collective_world"] == 2 and topo["distinct_devices"] == 1
    assert "rccl_world" not in topo and "not a multi-GPU measurement" in topo["note"]
    monkeypatch.setattr(torch, "ones", lambda *a, **k: torch.zeros(1, dtype=torch.int64))  # no GPU here
    with pytest.raises(SystemExit, match="distinct devices"):
        bench.rank_topology(2, 0, 0, "nccl", FakeDist(same, 2), args)
    two = [dict(same[0]), dict(same[1], device=1, pci="0000:05:00.0", uuid="GPU-bb")]
    topo = bench.rank_topology(2, 0, 0, "nccl", FakeDist(two, 2), args)
    assert topo["rccl_world"] == 2 and topo["distinct_devices"] == 2 and topo["backend"] == "rccl"
    with pytest.raises(SystemExit, match="RCCL counted 1 ranks"):
        bench.rank_topology(2, 0, 0, "nccl", FakeDist(two, 1), args)
    one = bench.rank_topology(1, 0, 0, "nccl", None, types.SimpleNamespace(gpus=1))
    assert one["collective_world"] == 1 and one["devices"][0]["pci"] == "0000:75:00.0"


def _run_bench(env_extra, *args):
    import subprocess

    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=300)


def test_bench_rejects_a_world_size_that_differs_from_gpus():
    r = _run_bench({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, "--gpus", "2", "--no-cpu")
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_bench_refuses_more_nccl_ranks_than_gpus():
    """Under nccl (RCCL) every rank needs its own GPU: asking for more exits non-zero with a
    message instead of silently running fewer ranks (here: no GPU at all)."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs visible")
    r = _run_bench({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "GDP_BENCH_BACKEND": "nccl"},
                   "--gpus", "2", "--no-cpu")
    assert r.returncode != 0 and "need 2 GPUs" in r.stderr


def test_traffic_records_match_only_their_kernel_instance():
    """roofline.traffic comes only from a PMC record of the same kernel instance: every build
    variant x tile order the autotune can pick has one on every config, and the convolution record
    is keyed by its conv kernel / rows / order."""
    import bench

    for cfg in ("c2", "c3", "c4", "c5"):
        for v in BUILD_VARIANTS:  # every variant the autotune can pick (20, 23, 27: contiguous spans)
            for t in (0, 1):
                for zw in (0, 1):  # the autotune also picks GDP_TUNE_ZERO_WINDOW
                    rec = bench.latest_pmc(cfg, v, t, zero_window=zw)
                    assert rec is not None and rec["variant"] == v and rec["tile_order"] == t, (cfg, v, t, zw)
                    assert rec.get("zero_window", 0) == zw, (cfg, v, t, zw)
                    assert rec.get("band_of") is None
                    # spans in the linear order re-read neighbouring units' decimated rows (<= 1.11x)
                    assert 0.99 < rec["kernel_bytes_per_launch"] / rec["algorithmic_bytes_per_launch"] < \
                        (1.12 if v >= 19 else 1.05), (cfg, v, t, zw)
    for n in (2, 4, 8):  # config 5 at N > 1: rank 0's band of N
        for v in BUILD_VARIANTS:
            for t in (0, 1):
                for zw in (0, 1):
                    rec = bench.latest_pmc("c5", v, t, zero_window=zw, band_of=n)
                    assert rec is not None and rec["band_of"] == n and rec["band_rows"][0] == 0, (n, v, t, zw)
                    assert rec["algorithmic_bytes_per_launch"] < bench.algorithmic_bytes(16384, 16384, 2, 5, 1) / n * 1.01
    assert bench.latest_pmc("c2", 99, 0) is None
    conv = bench.latest_conv_pmc("c2", {"conv_kernel": 2, "conv_rows": 32, "conv_order": 4})
    assert conv is not None and conv["op"] == "conv"
    for cfg in ("c2", "c4", "c5"):  # the round-3 default: 48-row block tiles
        rec = bench.latest_conv_pmc(cfg, {"conv_kernel": 2, "conv_rows": 48, "conv_order": 4})
        assert rec is not None and "k_conv_blk<5, 48, 16>" in rec["kernel"], cfg
    for cfg in ("c2", "c3", "c4", "c5"):  # the round-5 default: block order 5 (order 4 kept for one huge image)
        rec = bench.latest_conv_pmc(cfg, {"conv_kernel": 2, "conv_rows": 48, "conv_order": 5})
        # (round 6: the kernel gained its compile-time store pace, k_conv_blk<5, 48, 16, 2, 2>)
        assert rec is not None and re.search(r"k_conv_blk<5, 48, 16, 2(, 2)?>", rec["kernel"]), cfg
        assert 0.99 < rec["traffic_over_algorithmic"] < (1.15 if cfg == "c5" else 1.05), (cfg, rec["traffic_over_algorithmic"])
    assert bench.latest_conv_pmc("c2", {"conv_kernel": 0, "conv_rows": 16, "conv_order": 0}) is None


def test_subset_traffic_records_name_their_template_instance():
    """bench.py --op subset attaches PMC traffic only from a record of the subset build's own
    instance (op "subset", k_build<5, ..., true> for S = 2): never the full build's record of the
    same variant, nor another template instance's."""
    import bench

    rec = bench.latest_pmc("c2", 15, 0, "subset", 5)
    assert rec is not None and rec["op"] == "subset" and rec["kernel"].startswith("void (anonymous namespace)::k_build<5,")
    assert "true>" in rec["kernel"]  # the SUB template flag
    full = bench.latest_pmc("c2", 15, 0, "build", 5)
    assert full is not None and full["file"] != rec["file"]
    assert bench.latest_pmc("c2", 15, 0, "subset", 4) is None  # no k_build<0, ...> subset record


def test_inplace_traffic_records_name_their_block_shape():
    """bench.py --op regen / --op gauss attach PMC traffic only from a record of the same in-place
    kernel instance: every block shape the autotune can pick on config 2 has one,
    keyed by GDP_TUNE_INPLACE_SUB / _WINDOW_SUB, naming its template instance (configs 2 and 4)."""
    import bench

    for cfg, op, key, subs, kern in [(c, *x) for c in ("c2", "c4") for x in (
            ("regen", "inplace_sub", (1, 4, 2, 0, 8, 16, -16), "k_levels"), ("gauss", "window_sub", (1, 4, 2, 8, 16), "k_window"))]:
        for sub, zw in [(sub, zw) for sub in subs for zw in (0, 1)]:  # the autotune also picks the zero window
            rec = bench.latest_inplace_pmc(cfg, op, {key: sub, "zero_window": zw})
            assert rec is not None and rec["op"] == op and rec[key] == sub, (op, sub, zw)
            assert rec.get("zero_window", 0) == zw, (cfg, op, sub, zw)
            assert kern in rec["kernel"] and ("k_levels_x" in rec["kernel"]) == (op == "regen" and sub == 0)
            assert 0.99 < rec["kernel_bytes_per_launch"] / rec["algorithmic_bytes_per_launch"] < 1.05
            assert rec["bench_line_of_traced_run"]["parity"]["status"] == "bit-exact"
    assert bench.latest_inplace_pmc("c2", "regen", {"inplace_sub": 3}) is None
    assert bench.latest_inplace_pmc("c3", "gauss", {"window_sub": 4}) is None


def test_cpu_baseline_provenance_stamp(tmp_path):
    """cpu_baseline names the reference text its binary was compiled from:
    oracle/stamp.py records the sha256 of every source and of the binary; bench._ref_stamp copies it
    and re-hashes the binary it is about to run; a missing stamp is said, not papered over."""
    import subprocess

    import bench

    src = tmp_path / "GuassDePyramid.h"
    src.write_text("// stand-in source text for the stamp test\n")
    binary = tmp_path / "ref_avx512"
    binary.write_bytes(b"\x7fELF not really")
    assert "no stamp" in bench._ref_stamp(str(binary))["status"]
    subprocess.run([sys.executable, os.path.join(REPO, "oracle", "stamp.py"), str(binary), "g++", "-O2", str(src)],
                   check=True)
    st = bench._ref_stamp(str(binary))
    assert st["binary_matches_stamp"] is True and st["flags"] == "-O2"
    import hashlib

    assert st["sources_sha256"]["GuassDePyramid.h"] == hashlib.sha256(src.read_bytes()).hexdigest()
    binary.write_bytes(b"\x7fELF rebuilt without a new stamp")
    assert bench._ref_stamp(str(binary))["binary_matches_stamp"] is False


_LINE_PROBE = r"""
import json, os, sys, types
sys.path.insert(0, sys.argv[1])
import torch.distributed as dist
import bench
import __graft_entry__ as entry
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
dist.init_process_group("gloo", init_method="file://" + os.environ["GDP_BENCH_RDV"], rank=rank, world_size=world)
mg = __import__(entry.load_package().__name__ + ".distributed", fromlist=["sum_over_ranks"])
args = types.SimpleNamespace(steps=10, no_cpu=False, cpu_budget=0.2, op="build")
result = {"roofline": {"frac": 0.75}}
bytes_launch = 514_064_384 * (rank + 1)  # ranks may carry different shares (row bands)
bench.complete_line(result, args, rank, world, dist, mg, "cpu", bytes_launch, 10 * 0.1e-3)
if rank == 0:
    with open(sys.argv[2], "w") as f:
        json.dump(result, f)
dist.destroy_process_group()
"""


def test_multi_rank_line_carries_cpu_baseline_and_aggregate_roofline(tmp_path):
    """at N > 1 the line still carries `cpu_baseline` (rank 0 samples it after
    every rank's timed region while the others wait at a barrier) and the whole-job
    `frac_aggregate` = sum of every rank's algorithmic bytes / ms_per_step / (N x 8 TB/s) —
    two self-launched gloo ranks (bench.launch_ranks, the driver's --gpus N path) through the
    same bench.complete_line the GPU run calls."""
    import json

    import bench

    probe = tmp_path / "probe.py"
    probe.write_text(_LINE_PROBE)
    out = tmp_path / "line.json"
    assert bench.launch_ranks(2, [REPO, str(out)], script=str(probe)) == 0
    line = json.loads(out.read_text())
    total = 514_064_384 * 3
    assert line["roofline"]["aggregate_bytes_per_step"] == total
    assert line["roofline"]["frac_aggregate"] == round(total / 0.1e-3 / (2 * 8000e9), 4)
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["unit"] == "Mpix/s" and cb["cores"] >= 1 and cb["kind"] in ("reference", "port")
    assert "after all 2 ranks finished their timed steps" in cb["when"]


def test_serving_figure_is_opt_in():
    """`concurrent_streams` overlaps launches of the bench's own kernel instance; it must stay out of
    the default command (whose `rocprofv3 --stats` average the judge compares with `kernel_ms`) and
    run before the warm-up, so the timed launches remain the last ones on the bench's stream."""
    import re

    src = open(os.path.join(REPO, "bench.py")).read()
    assert re.search(r'"--concurrent-streams", type=int, default=0', src)
    main = src[src.index("def main():"):]
    assert main.index("concurrent_streams(ctxs") < main.index("for _ in range(args.warmup):")
