"""T3 rehearsal of the multi-GPU DDP path on ONE MI355X (several ranks share GPU 0; gloo process
group for bootstrap, the direct xGMI all-reduce kernels for the gradients - RCCL cannot put two ranks
on one GPU, so these runs need none):

* W ranks on disjoint shards == the world-1 engine on the concatenated batch (tools/ddp_equivalence.py);
* ``mnist_ddp.py`` end to end at world 2 on the fused engine: rank-0-only train / test lines, the
  ``world * batch_idx * len(data)`` sample counter, ``module.``-prefixed checkpoint, ``--check-sync``,
  a ``Total cost time`` line per rank (reference mnist_ddp.py:74-79, :161-203);
* ``bench.py --gpus 2`` under torchrun: the JSON proves correctness, not just speed (params_in_sync,
  the all-reduce used, the reference-script total_cost_time_s)."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    # several ranks on one GPU: 2 hardware queues per process (docs/DEBUGGING.md, queue oversubscription)
    return dict(os.environ, PYTHONPATH=ROOT, MNIST_AMD_ONE_GPU="1", GPU_MAX_HW_QUEUES="2", **kw)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ddp_matches_world1_large_batch(gpu_box, world):
    # W*B stays below FC1_BIG_MIN_B (512) so the world-1 run on the W*B batch uses the same forward
    # kernels as the shards: the forward is then row-wise bitwise identical and only the gradient
    # reductions differ in order (at W*B >= 512 fc1 switches to its 4-way split-K form, whose
    # different rounding of every row's z1 flips bf16 ties in h / dz1 - a legitimate but larger
    # difference than the summation-order noise floor samples)
    B = {2: 200, 4: 100, 8: 60}[world]
    cmd = [sys.executable, "-u", os.path.join(ROOT, "tools", "ddp_equivalence.py"), "--world", str(world),
           "--same-device", "--steps", "10", "--batch", str(B), "--timeout", "260"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=_env())
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "DDP_EQUIVALENCE PASS" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("W", [2, 8])
def test_mnist_ddp_xgmi_without_rccl(gpu_box, tmp_path, W):
    n_train, B = 8000, 200 if W == 2 else 50       # 20 steps per rank per epoch either way
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes", "1", "--nproc-per-node", str(W), os.path.join(ROOT, "mnist_ddp.py"),
           "--batch-size", str(B), "--epochs", "2", "--synthetic", "--synthetic-train-size", str(n_train),
           "--synthetic-test-size", "1000", "--dist-backend", "gloo", "--allreduce", "xgmi", "--check-sync",
           "--save-model", "--json-log", str(tmp_path / "log.jsonl")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=tmp_path, env=_env())
    out = r.stdout
    assert r.returncode == 0, (out[-3000:], r.stderr[-3000:])
    # every rank prints its init line and the timer; only rank 0 prints train / test lines
    assert len(re.findall(r"\| distributed init \(rank \d\): env://", out)) == W
    assert len(re.findall(r"Total cost time:[0-9.]+ ms", out)) == W
    train = re.findall(r"Train Epoch: (\d+) \[(\d+)/(\d+) \((\d+)%\)\]\tLoss: ([0-9.]+)", out)
    steps = n_train // W // B                                   # 20 per rank per epoch
    assert len(train) == 2 * len(range(0, steps, 10))           # rank 0 only, every 10 batches
    assert [int(t[1]) for t in train[:2]] == [0, W * 10 * B]    # world * batch_idx * len(data)
    assert all(int(t[2]) == n_train for t in train)
    assert len(re.findall(r"Test set: Average loss: [0-9.]+, Accuracy: \d+/1000", out)) == 2
    import torch
    sd = torch.load(tmp_path / "mnist_cnn.pt", map_location="cpu", weights_only=True)
    assert sorted(sd) == sorted("module." + k for k in ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias",
                                                        "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"))
    assert all(v.dtype == torch.float32 for v in sd.values())
    # the startup inside the reference timer, per phase and per rank (--json-log "setup_s")
    import json
    recs = [json.loads(ln) for ln in open(tmp_path / "log.jsonl")]
    setups = [x for x in recs if "setup_s" in x]
    assert len(setups) == W and all(x["allreduce"] == "xgmi" for x in setups)
    for x in setups:
        assert {"pg_init", "data", "ddp_wrap", "trainer.xgmi_comm", "trainer.validate.xgmi"} <= set(x["setup_s"])
        assert not any(k.startswith("rccl") for k in x["setup_s"])   # --allreduce xgmi: no RCCL communicator
        assert x["transport_report"]["xgmi"]["ok"] and x["transport_report"]["xgmi"]["us_per_step"] > 0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("W,launcher", [(2, "torchrun"), (8, "self")])
def test_bench_reports_correctness(gpu_box, tmp_path, W, launcher):
    """``bench.py --gpus W`` under torchrun, and (W = 8) launching its W ranks itself with no launcher
    (the driver's plain command): ONE JSON line with n_gpus W, params in sync, the transport, its
    validation and the per-phase setup seconds."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(W), "--steps", "20", "--warmup", "5", "--epochs", "2",
            "--dist-backend", "gloo", "--allreduce", "xgmi"] + (["--no-script-run"] if W > 4 else [])
    # (W ranks + a W-rank child job would hold 2W processes on the one GPU; the box allows 16)
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
               "--nnodes", "1", "--nproc-per-node", str(W)] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=tmp_path, env=_env())
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j["n_gpus"] == W and j["params_in_sync"] is True and j["desync_epoch"] is None
    assert j["config"]["allreduce"] == "xgmi" and j["config"]["rccl_world"] is None
    assert j["config"]["rccl_comms"] == 0 and j["config"]["xgmi_ordering"].startswith("uncached")
    assert j["config"]["xgmi_validation"].startswith("ok (graph replay")
    assert j["config"]["transport_report"]["xgmi"]["us_per_step"] > 0
    assert "trainer.validate.xgmi" in j["setup_phases_s"] and "warm_replay" in j["setup_phases_s"]
    if launcher == "self":
        assert j["launcher"]["child_rc"] == 0 and j["launcher"]["kind"].startswith("bench.py self-launch")
    if W <= 4:
        rs = j["reference_script"]
        assert rs["rc"] == 0 and rs["ranks_reporting"] == W, rs
        assert j["total_cost_time_s"] > 0 and rs["setup_phases_s"]["pg_init"] >= 0


@pytest.mark.timeout(200)
def test_validation_fault_in_replayed_graph_is_named(gpu_box, tmp_path):
    """A rank held back while the startup validation REPLAYS the captured training graph: its peers'
    stage waits time out inside the graph, the collective verdict names the ranks, and with no RCCL
    communicator to fall back to (gloo + --allreduce xgmi) the run stops with that error instead of
    training on a poisoned communicator."""
    W = 4
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes", "1", "--nproc-per-node", str(W), os.path.join(ROOT, "mnist_ddp.py"),
           "--batch-size", "100", "--epochs", "1", "--synthetic", "--synthetic-train-size", "4000",
           "--synthetic-test-size", "1000", "--dist-backend", "gloo", "--allreduce", "xgmi"]
    env = _env(MNIST_AMD_FAULT="validate_delay:2:6", MNIST_AMD_STARTUP_TIMEOUT="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=tmp_path, env=env)
    err = r.stdout + r.stderr
    assert r.returncode != 0, err[-3000:]
    assert "no gradient all-reduce passed its startup validation" in err, err[-3000:]
    assert "[xgmi] startup validation failed" in err and "timed out" in err and "rank 2" in err, err[-3000:]
    assert "Train Epoch" not in r.stdout                         # nothing trained on the bad comm


@pytest.mark.timeout(200)
def test_bench_startup_fault_reports_json(gpu_box, tmp_path):
    """The same fault through ``bench.py --gpus 4`` (self-launched ranks): rank 0 still prints ONE
    JSON line - value null, the failing phase, the decoded error and every rank's failure record
    with its transport report and setup phases - and the exit code is non-zero."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "20", "--warmup", "5",
           "--no-full-run", "--dist-backend", "gloo", "--allreduce", "xgmi", "--batch-size", "100"]
    env = _env(MNIST_AMD_FAULT="validate_delay:2:6", MNIST_AMD_STARTUP_TIMEOUT="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=tmp_path, env=env)
    assert r.returncode != 0, r.stdout[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    j = json.loads(lines[0])
    assert j["value"] is None and j["n_gpus"] == 4 and j["failed_phase"] == "trainer"
    assert "no gradient all-reduce passed its startup validation" in j["error"]
    assert "timed out" in j["error"]
    recs = j["rank_failures"]
    assert "0" in recs and len(recs) >= 2, recs.keys()
    r0 = recs["0"]
    assert {"pg_init", "data_model", "trainer.xgmi_comm", "trainer.validate.xgmi"} <= set(r0["setup_phases_s"])
    assert r0["transport_report"]["xgmi"]["ok"] is False and "timed out" in r0["transport_report"]["xgmi"]["validation"]
    assert j["launcher"]["child_rc"] != 0


@pytest.mark.timeout(200)
def test_bench_nccl_process_group_stays_lazy_w4(gpu_box, tmp_path):
    """Production bootstrap on one GPU: the default ``nccl`` process group (lazy - no device_id) with
    the xGMI transport.  RCCL refuses two ranks on one GPU, so this passes only if nothing in the
    fused path issues a torch collective (ProcessGroupNCCL would build a communicator): shape check,
    broadcast (over the xGMI mappings), verdicts, timing maxima and fingerprints all go over the
    TCPStore."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "20", "--warmup", "5",
           "--no-full-run", "--allreduce", "xgmi"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=tmp_path, env=_env())
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    j = json.loads(lines[-1])
    assert j["n_gpus"] == 4 and j["params_in_sync"] is True and j["config"]["allreduce"] == "xgmi"
    assert "pg_init" in j["setup_phases_s"] and j["config"]["rccl_comms"] == 0


@pytest.mark.timeout(300)
def test_mnist_ddp_stdout_contract_nccl_check_sync_w2(gpu_box, tmp_path):
    """``mnist_ddp.py`` at world 2 on the production ``nccl`` process group (lazy) with ``--check-sync``:
    rank 0's stdout holds only the reference's line kinds (init line, train lines, test
    lines, the timer - the transport line goes to stderr), and the per-epoch desync check runs over
    the store: RCCL refuses two ranks on one GPU, so a torch collective on the nccl group (which
    would build ProcessGroupNCCL's communicator) fails this test."""
    W, n_train, B = 2, 8000, 200
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes", "1", "--nproc-per-node", str(W), os.path.join(ROOT, "mnist_ddp.py"),
           "--batch-size", str(B), "--epochs", "2", "--synthetic", "--synthetic-train-size", str(n_train),
           "--synthetic-test-size", "1000", "--allreduce", "xgmi", "--check-sync"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=tmp_path, env=_env())
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    kinds = (r"\| distributed init \(rank \d\): env://, local rank:\d, world size:2",
             r"Train Epoch: \d+ \[\d+/\d+ \(\d+%\)\]\tLoss: [0-9.]+",
             r"Test set: Average loss: [0-9.]+, Accuracy: \d+/\d+ \(\d+%\)",
             r"Total cost time:[0-9.eE+-]+ ms", r"")
    bad = [ln for ln in r.stdout.splitlines() if not any(re.fullmatch(k, ln) for k in kinds)]
    assert not bad, bad[:10]
    assert len(re.findall(r"Test set: Average loss", r.stdout)) == 2
    assert "| gradient all-reduce: xgmi" in r.stderr


@pytest.mark.timeout(300)
@pytest.mark.parametrize("W", [2, 8])
def test_bench_fp32_xgmi_rehearsal(gpu_box, tmp_path, W):
    """The fp32 step (the reference's precision) on the xGMI transport: ``bench.py --dtype fp32`` at
    W ranks on one GPU (gloo + --allreduce xgmi, no RCCL) trains with every rank's parameters bitwise
    equal, validated by replaying the captured fp32 chunk."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(W), "--steps", "10", "--warmup", "2",
           "--no-full-run", "--dist-backend", "gloo", "--allreduce", "xgmi", "--dtype", "fp32",
           "--batch-size", "64", "--graph-steps", "5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=tmp_path, env=_env())
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert j["n_gpus"] == W and j["dtype"] == "fp32" and j["params_in_sync"] is True
    assert j["config"]["allreduce"] == "xgmi" and j["config"]["schedule"] == "xgmi"
    assert j["config"]["xgmi_validation"].startswith("ok (graph replay")


def _driver_cmd(W, tmp_path, *extra, n_train=8000, B=200, epochs=2):
    return [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
            "--nnodes", "1", "--nproc-per-node", str(W), os.path.join(ROOT, "mnist_ddp.py"),
            "--batch-size", str(B), "--epochs", str(epochs), "--synthetic", "--synthetic-train-size", str(n_train),
            "--synthetic-test-size", "1000", "--json-log", str(tmp_path / "log.jsonl"), *extra]


def _setups(tmp_path):
    return [x for x in (json.loads(ln) for ln in open(tmp_path / "log.jsonl")) if "setup_s" in x]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("W", [2, 4])
def test_production_command_trains_on_xgmi_rccl_never_waited(gpu_box, tmp_path, W):
    """The driver's PRODUCTION command - default ``nccl`` process group, default ``--allreduce auto``, no
    transport flag - with W ranks sharing GPU 0 (where RCCL could not initialise: two ranks on one
    GPU): the xGMI transport validates first, RCCL is never started or waited for (no rccl phase
    inside the reference timer), the run trains and exits 0."""
    r = subprocess.run(_driver_cmd(W, tmp_path), capture_output=True, text=True, timeout=280, cwd=tmp_path,
                       env=_env())
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert len(re.findall(r"Total cost time:[0-9.]+ ms", r.stdout)) == W
    assert len(re.findall(r"Test set: Average loss", r.stdout)) == 2
    setups = _setups(tmp_path)
    assert len(setups) == W
    for x in setups:
        assert x["allreduce"] == "xgmi", x["transport_report"]
        rep = x["transport_report"]
        assert rep["xgmi"]["ok"] and rep["rccl"]["ok"] is None, rep
        assert rep["rccl"]["validation"].startswith("not needed") and "not started" in rep["rccl"]["validation"]
        assert not any(k.startswith("trainer.rccl") or k.startswith("rccl_comm_wait") for k in x["setup_s"]), x["setup_s"]


@pytest.mark.timeout(300)
def test_fastest_drops_failed_rccl_init_and_keeps_xgmi(gpu_box, tmp_path):
    """``--allreduce fastest`` starts RCCL's non-blocking init at once; with two ranks on one GPU it
    fails (or is cut off by its init timeout): the failure drops the RCCL candidate on every rank
    (collective) instead of ending the run, the validated xGMI schedule trains, and the transport
    report names the init failure."""
    r = subprocess.run(_driver_cmd(2, tmp_path, "--allreduce", "fastest"), capture_output=True, text=True,
                       timeout=280, cwd=tmp_path, env=_env(MNIST_AMD_RCCL_INIT_TIMEOUT="40"))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    for x in _setups(tmp_path):
        rep = x["transport_report"]
        assert x["allreduce"] == "xgmi" and rep["xgmi"]["ok"], rep
        assert rep["rccl"]["ok"] is False and "RCCL communicator init failed" in rep["rccl"]["validation"], rep


@pytest.mark.timeout(300)
def test_auto_falls_back_to_rccl_when_xgmi_fails(gpu_box, tmp_path):
    """``--allreduce auto`` where the xGMI validation fails (rank 1 held back past the stage timeout):
    only then is RCCL brought up - here it cannot initialise (two ranks on one GPU) - and the run stops
    with ONE error naming both candidates' failures instead of hanging."""
    env = _env(MNIST_AMD_FAULT="validate_delay:1:6", MNIST_AMD_STARTUP_TIMEOUT="2", MNIST_AMD_RCCL_INIT_TIMEOUT="40")
    r = subprocess.run(_driver_cmd(2, tmp_path, epochs=1), capture_output=True, text=True, timeout=280,
                       cwd=tmp_path, env=env)
    err = r.stdout + r.stderr
    assert r.returncode != 0, err[-3000:]
    assert "no gradient all-reduce passed its startup validation" in err, err[-3000:]
    assert "xgmi:" in err and "rccl:" in err and "RCCL communicator init failed" in err, err[-3000:]
    assert "Train Epoch" not in r.stdout
