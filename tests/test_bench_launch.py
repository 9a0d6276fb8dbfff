"""bench.py's multi-rank launch contract on the CPU (gloo, no device work):
`python bench.py --gpus 2` spawns its own two ranks (no launcher), and the
torch.distributed.run launch the driver uses reaches the same code; either way
rank 0 prints one JSON line with n_gpus 2 and the reference's global batch split
over the ranks (C3 global 65,536)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _json_line(out):
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["NCF_SAMPLER_THREADS"] = "2"
    return env


def test_bench_spawns_its_own_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-harness",
                        "--config", "c3"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2
    assert d["config"]["global_batch"] == 65536 and d["config"]["per_gpu_batch"] == 32768
    assert d["config"]["parallelism"] == "dp2" and d["value"] > 0 and "harness" in d


def test_bench_under_torch_distributed_run():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-harness", "--config", "c2"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 1024 and d["config"]["per_gpu_batch"] == 512


def test_failed_rank_stops_the_others():
    """A rank that dies after the rendezvous makes the spawner stop the rest (rank 0
    would wait in a collective forever) and exit non-zero."""
    env = _env()
    env["NCF_BENCH_FAIL_RANK"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-harness",
                        "--config", "c3"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_roofline_traffic_sources_in_committed_profiles():
    """Every bench config's roofline finds its counter traffic in a committed
    rocprofv3 summary: the fused path by its launch group's kernel names, the layered
    path (CLI, stress) by every kernel of its step weighted per step."""
    sys.path.insert(0, ROOT)
    import bench
    t, busy, src = bench.layered_profile("stress")
    assert src is not None and t > 1e9 and 0 < busy < 1, (t, busy, src)
    # weights per step: one launch each per step of the projection (the step's first),
    # the wide step chain and the weight-gradient launch (round 6; the per-layer GEMM
    # launches of earlier profiles counted per layer)
    d = json.load(open(os.path.join(ROOT, src)))
    ks = {k["kernel"]: k for k in d["kernels"]}
    proj = [k for n, k in ks.items() if n.startswith("ncf::lyr_proj_kernel")]
    assert len(proj) == 1
    for name in ("ncf::lyr_wide_chain_kernel", "ncf::lyr_bwd_w_multi_kernel<128>"):
        assert ks[name]["calls"] == proj[0]["calls"], name
    assert bench.layered_profile("cli")[0] is not None
    tr, src3 = bench.pmc_traffic("c3", ["ncf::ncf_step_kernel<16, 3, 2, false, true, 8>",
                                        "ncf::fact_expand_kernel<64>"])
    assert tr is not None and tr > 1e6, src3
