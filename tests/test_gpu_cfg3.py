"""BASELINE config 3 on one device: the exact 8-rank strong-scaling split of
the 1024 x 1024 p = 8 mesh (1,048,576 elements, 67,125,249 DOF; 8 strips of
128 x 1024 elements) that the driver's 8-GPU run executes, with every rank on
cuda:0 (RCCL refuses two ranks on one GPU, so the interface sum travels over
the torch/gloo callback transport; every other part of each rank's step is
the production sem_dd path: interface elements on the side stream, pack,
exchange, fused finish).

Checks (the serial loop replaced is
/root/reference/sem/discrete.py:208-209):
* ranks_seen == 8, each rank 131,072 elements;
* every rank's 2-column block in the middle of its strip <= 1e-10 relative
  L2 against the NumPy oracle of the reference path;
* every rank's own side of the two element columns across its right
  interface <= 1e-10 against the oracle (the shared node line only holds the
  global value after the exchange);
* every interface node of every rank equals the single-GPU action of the
  whole mesh (same global u) to 1e-12 relative (only the summation order of
  the shared entries differs).

Also the timing-only mode (bench.py --time-rank): one interior rank of the
8-strip split alone on the GPU through the loopback transport -- the JSON
must carry the step, interior-alone and side-chain times and the host split.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _bench(args, timeout):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


@pytest.mark.timeout(900)
def test_cfg3_eight_strips_on_one_gpu(gpu, tmp_path):
    res, err = _bench(["--gpus", "8", "--rehearse-one-gpu", "--steps", "3", "--warmup", "1",
                       "--no-cpu-baseline", "--dump-interface", str(tmp_path),
                       "--deadline", "700"], timeout=800)
    cfg = res["config"]
    assert cfg["ranks_seen"] == 8 and res["n_gpus"] == 8
    assert cfg["n_elem_global"] == 1024 * 1024 and cfg["n_elem_per_gpu"] == 128 * 1024
    assert cfg["ndof_global"] == 67125249
    pr = res["parity_per_rank"]
    assert len(pr) == 8 and all(e < 1e-10 for e in pr), pr
    pi = res["parity_interface_per_rank"]
    assert len(pi) == 8 and pi[7] is None
    assert all(e is not None and e < 1e-10 for e in pi[:7]), pi
    print("cfg3 8 strips: block parity per rank", pr, "interface parity", pi)

    # every rank's interface node lines against the single-GPU action of the
    # whole mesh on the same global u
    sys.path.insert(0, ROOT)
    from bench import global_random_field
    from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
    part = StripPartition(1024, 1024, 8, 1, 0)
    nodes, e2n = part.local_mesh(0.05)
    op = OverlappedOperator(8, nodes, e2n, {}, 1, gpu, world=1, rank=0)
    del nodes, e2n
    u = global_random_field(part, 1, 0, op.ndof, gpu)
    y = op.apply(u)
    worst, n_checked = 0.0, 0
    for r in range(8):
        d = np.load(tmp_path / ("iface_rank%d.npz" % r))
        gid = torch.from_numpy(d["gid"].astype(np.int64)).to(gpu)
        ref = y[gid].cpu().numpy()
        assert d["y"].size == (1 if r in (0, 7) else 2) * (1024 * 8 + 1)
        err = np.linalg.norm(d["y"] - ref) / np.linalg.norm(ref)
        worst = max(worst, err)
        n_checked += ref.size
    op.close()
    print("interface nodes vs single GPU: %d values, worst rank rel-L2 %.2e" % (n_checked, worst))
    assert worst < 1e-12


@pytest.mark.timeout(600)
@pytest.mark.parametrize("transport", ["rccl_self", "loopback"])
def test_time_rank(gpu, transport):
    """One interior rank (two peers) of the 8-strip split timed alone, the
    exchange as RCCL send/recv to itself or the loopback copy; the values are
    meaningless by construction, the structure of the report is what is
    checked here (the numbers are measured by the GPU calls and kept under
    profiles/)."""
    res, _ = _bench(["--gpus", "8", "--time-rank", "3", "--steps", "10", "--warmup", "3",
                     "--time-rank-transport", transport], timeout=500)
    assert res["transport"] == transport
    assert res["rank"] == 3 and res["of_ranks"] == 8 and res["peers"] == [2, 4]
    assert res["strip_elements"] == "128 x 1024"
    for k in ("step", "interior_alone", "side_chain_alone", "single_gpu_whole_mesh"):
        assert res[k]["event_ms_avg"] > 0, k
    assert res["host"]["host_us_per_apply"] > 0
    assert res["interface_elements"] == 2 * 1024
    print(json.dumps(res))
