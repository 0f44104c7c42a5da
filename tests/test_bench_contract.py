"""bench.py contract on CPU: launched like the driver's multi-GPU run (torch.distributed.run, 2
gloo ranks, rendezvous on 127.0.0.1), rank 0 prints exactly ONE JSON line with the required keys and
the whole-job aggregate."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    from heat_amd.run import free_port

    return free_port()


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


import pytest


@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_multi_rank_one_json_line(ranks):
    env = dict(os.environ, HEAT_COMM_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks), "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(ranks), "--steps", "2", "--warmup", "1",
           "--n-per-gpu", "3000", "--exact-steps", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    rec = lines[0]
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == ranks and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["scaling"] == "weak" and rec["higher_is_better"] is True
    assert rec["config"]["global_batch"] == 3000 * ranks and rec["config"]["parallelism"] == "dp%d" % ranks
    assert rec["extra"]["world_size_seen_by_rccl"] == ranks
    # self-validation of the distributed step (outside the timed region)
    assert rec["extra"]["centroids_agree"] is True
    assert rec["extra"]["count_sum_ok"] is True
    assert rec["extra"]["centroid_max_rel_err_vs_fp64"] < 1e-5
    assert rec["extra"]["allreduce_us"] > 0
    # the labels are the fp64 argmin (sampled on every rank)
    assert rec["extra"]["labels_checked"] == 3000 * ranks
    assert rec["extra"]["labels_ok"] is True and rec["extra"]["label_max_excess"] <= 4e-6
    assert rec["extra"]["label_agreement"] > 0.999
    # whole-job aggregate: 2 n k f flops per step over the max-over-ranks step time
    flops = 2 * 3000 * ranks * 1024 * 64
    assert abs(rec["value"] - flops / (rec["ms_per_step"] * 1e-3) / 1e9) <= 1e-6 * rec["value"]


@pytest.mark.parametrize("workload", ["moments", "cdist", "knn", "qr"])
def test_bench_secondary_workloads_validate(workload):
    env = dict(os.environ, HEAT_COMM_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    extra_args = {"moments": ["--n-per-gpu", "100000"], "qr": ["--n-per-gpu", "3000", "--f", "48"]}.get(
        workload, ["--rows", "6000", "--f", "8"])
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--workload", workload] + extra_args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    ex = lines[0]["extra"]
    if workload == "moments":
        assert ex["mean_abs_err_vs_fp64"] < 1e-5 and ex["var_rel_err_vs_fp64"] < 1e-5
    elif workload == "cdist":
        assert ex["sample_max_sq_err_rel_vs_fp64"] < 1e-5
    elif workload == "qr":
        assert lines[0]["scaling"] == "weak" and lines[0]["config"]["global_batch"] == 6000
        assert ex["qr_ok"] is True and ex["q_orth_err_64cols"] < 1e-5 and ex["r_upper"] is True
    else:
        assert lines[0]["scaling"] == "strong" and lines[0]["config"]["global_batch"] == 6000
        assert ex["self_first"] is True and ex["index_agreement"] == 1.0 and ex["max_rel_dist_err"] < 1e-5


def _clean_env(**kw):
    env = dict(os.environ, HEAT_COMM_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", **kw)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        if k not in kw:
            env.pop(k, None)
    return env


def test_bench_self_launches_gpus_ranks():
    """``bench.py --gpus 4`` with no launcher starts 4 rank processes itself and relays ONE JSON
    line from rank 0 that saw a 4-rank device world."""
    cmd = [sys.executable, "bench.py", "--gpus", "4", "--steps", "2", "--warmup", "1", "--n-per-gpu", "3000",
           "--exact-steps", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=_clean_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    rec = lines[0]
    assert rec["n_gpus"] == 4 and rec["extra"]["world_size_seen_by_rccl"] == 4
    assert rec["config"]["parallelism"] == "dp4" and rec["config"]["global_batch"] == 4 * 3000
    # every path the run took is recorded, and the A/B all-reduce timing ran and was checked
    assert rec["extra"]["comm"]["collective_paths"].get("allreduce:pg", 0) > 0
    ab = rec["extra"]["comm_ab"]
    assert ab["pg_8B_ok"] is True and ab["pg_532480B_ok"] is True and ab["pg_8B_us"] > 0


def test_bench_world_size_mismatch_fails():
    cmd = [sys.executable, "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=_clean_env(WORLD_SIZE="2", RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert not _json_lines(r.stdout)


def test_bench_failing_rank_fails_the_job():
    """A rank that dies (here: an invalid workload size on every rank) makes the self-launched job
    exit non-zero without a JSON line."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--n-per-gpu", "-5"]
    r = subprocess.run(cmd, cwd=ROOT, env=_clean_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)


def test_check_labels_catches_a_wrong_assignment():
    """bench.check_labels: the argmin labels pass; labels with 1 % of the points moved to a far
    centroid fail (a wrong assign kernel would pass the centroid checks, which reuse its labels)."""
    import torch

    sys.path.insert(0, ROOT)
    import bench
    from heat_amd.core.communication import MPI_WORLD

    g = torch.Generator().manual_seed(0)
    X = torch.randn(20000, 16, generator=g)
    C = torch.randn(64, 16, generator=g)
    lab = torch.cdist(X.double(), C.double()).argmin(1)
    ok = bench.check_labels(X, C, lab, MPI_WORLD, sample=4096)
    assert ok["labels_ok"] and ok["label_agreement"] == 1.0 and ok["labels_checked"] == 4096
    far = torch.cdist(X.double(), C.double()).argmax(1)
    bad = torch.where(torch.arange(20000) % 100 == 0, far, lab)
    res = bench.check_labels(X, C, bad, MPI_WORLD, sample=20000)
    assert not res["labels_ok"] and res["label_max_excess"] > 1e-2
    assert abs(res["label_agreement"] - 0.99) < 1e-3


def test_bench_shared_gpu_rehearsal_records_itself():
    """HEAT_BENCH_SHARED_GPU=1: the N-rank job runs on a gloo world whatever the device count and
    the record says shared_gpu (never a scaling point)."""
    cmd = [sys.executable, "bench.py", "--gpus", "3", "--steps", "1", "--warmup", "1", "--n-per-gpu", "2000",
           "--exact-steps", "0", "--comm-ab", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=_clean_env(HEAT_BENCH_SHARED_GPU="1"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["config"]["shared_gpu"] is True and rec["extra"]["shared_gpu"] is True
    assert rec["extra"]["world_size_seen_by_rccl"] == 3 and rec["extra"]["labels_ok"] is True
