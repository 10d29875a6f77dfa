"""Multi-GPU sharding of one stack on the CPU: the slab
plan, the slab join (lfm_merge_slabs in liblfm, no GPU needed) against the
oracle's one-piece encode, and the bench's world-size-2 rank protocol over
gloo (selection on the stack's frame 0 on every rank, one slab per rank, an
all_gather of slab sizes, every rank placing its blocks into one shared
.lfm with lfm_place_slab, MAX-over-ranks timing).  The slabs here come from
the oracle (no GPU); tests/test_multigpu_gpu.py runs the same protocol with
the product encoder on the GPU."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import REPO
from lfm.shard import forced_request, plan_slabs


def test_plan_slabs_properties():
    for Z in (1, 7, 8, 20, 64, 256, 257):
        for world in (1, 2, 3, 4, 8):
            for bz in (1, 4, 8):
                plan = plan_slabs(Z, world, bz)
                assert len(plan) == world
                z = 0
                for i, (z0, d) in enumerate(plan):
                    assert z0 == z and d >= 0
                    z += d
                    last_nonempty = all(dd == 0 for _, dd in plan[i + 1:])
                    if d and not last_nonempty:
                        assert d % bz == 0
                assert z == Z
    assert plan_slabs(256, 8, 8) == [(32 * r, 32) for r in range(8)]
    with pytest.raises(ValueError):
        plan_slabs(0, 2)
    assert forced_request(4, True) == 0x8C and forced_request(0) == 8


def _slabs(oracle, img, world, bz, hv, fam, bs):
    out = []
    for z0, d in plan_slabs(img.shape[2], world, bz):
        if d:
            prev = img[0, 0, z0 - 1] if z0 else None
            out.append(oracle.encode(img[:, :, z0:z0 + d], header_version=hv, nnum=13, family=fam, block_size=bs,
                                     z0=z0, prev=prev))
    return out


@pytest.mark.parametrize("fam,video,Z,world,bz", [("tiles", True, 20, 3, 4), ("angle", False, 16, 2, 8),
                                                  ("space", False, 9, 4, 2), ("tiles", True, 11, 2, 1)])
def test_merge_slabs_equals_one_piece(lfmlib, oracle, fam, video, Z, world, bz):
    img = oracle.synthetic_lf(70, 45, Z=Z, T=13, seed=Z * 31 + world)
    k, _ = oracle.select(img[0, 0, 0], 13, fam)
    bs = [32, 16, bz, 1, 1]
    full = oracle.encode(img, header_version=(0x80 if video else 0), nnum=13, family=fam, block_size=bs)
    slabs = _slabs(oracle, img, world, bz, forced_request(k, video), fam, bs)
    assert lfmlib.merge_slabs(slabs) == full


def test_merge_slabs_rejects_mismatch(lfmlib, oracle):
    img = oracle.synthetic_lf(70, 45, Z=16, T=13, seed=3)
    bs = [32, 16, 8, 1, 1]
    a = oracle.encode(img[:, :, :8], header_version=8 + 4, nnum=13, family="tiles", block_size=bs)
    b = oracle.encode(img[:, :, 8:], header_version=8 + 3, nnum=13, family="tiles", block_size=bs, z0=8)
    with pytest.raises(lfmlib.LfmError):
        lfmlib.merge_slabs([a, b])  # different predictors
    c = oracle.encode(img[:, :, :6], header_version=8 + 4, nnum=13, family="tiles", block_size=bs)
    d = oracle.encode(img[:, :, 6:], header_version=8 + 4, nnum=13, family="tiles", block_size=bs, z0=6)
    with pytest.raises(lfmlib.LfmError):
        lfmlib.merge_slabs([c, d])  # first slab not a whole number of blocks deep
    assert lfmlib.merge_slabs([a]) == a


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, result_path):
    import sys
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "lightfieldmicroscopy_pc-bzip2_amd"), os.path.join(repo, "oracle")):
        sys.path.insert(0, p)
    import bench
    import lfm_oracle as O
    from lfm.shard import forced_request, max_over_ranks, plan_slabs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shm = None
    try:
        Z, fam, bs = 24, "tiles", [32, 16, 8, 1, 1]
        img = O.synthetic_lf(64, 40, Z=Z, T=13, seed=0x4C464D04)  # every rank regenerates the stack (synthetic)
        k, _ = O.select(img[0, 0, 0], 13, fam)  # the stack's frame 0, redundantly on every rank
        z0, d = plan_slabs(Z, world, 8)[rank]
        slab = O.encode(img[:, :, z0:z0 + d], header_version=forced_request(k, True), nnum=13, family=fam,
                        block_size=bs, z0=z0, prev=img[0, 0, z0 - 1] if z0 else None)
        shm = bench.SharedLfm(rank, world, 1 << 22)
        bench.place_in_shared(shm, slab, rank, world, Z, "gloo", 2)
        dist.barrier()
        t = max_over_ranks(0.25 * (rank + 1))
        if rank == 0:
            merged = bytes(shm.buf[:shm.len])
            full = O.encode(img, header_version=0x80, nnum=13, family=fam, block_size=bs)
            with open(result_path, "w") as f:
                f.write("%d %.3f" % (int(merged == full), t))
        dist.barrier()
    finally:
        if shm is not None:
            shm.close()
        dist.destroy_process_group()


def test_gloo_two_rank_sharded_encode(tmp_path):
    import torch.multiprocessing as mp
    res = tmp_path / "res.txt"
    mp.spawn(_rank_main, args=(2, _free_port(), str(res)), nprocs=2, join=True)
    ok, t = res.read_text().split()
    assert ok == "1"
    assert float(t) == pytest.approx(0.5)


_LAUNCH_VARS = ("LFM_GPUS", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_SIZE",
                "OMPI_COMM_WORLD_LOCAL_RANK")


@pytest.mark.parametrize("env,nvis,current,want", [
    ({}, 8, 0, list(range(8))),                                       # plain process: every GPU
    ({"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8", "LOCAL_RANK": "3"}, 8, 0, [3]),  # torchrun rank 3
    ({"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "1", "LOCAL_RANK": "0"}, 8, 0, list(range(8))),  # 1 proc per node
    ({"WORLD_SIZE": "16", "LOCAL_WORLD_SIZE": "8", "LOCAL_RANK": "11"}, 8, 0, [3]),  # modulo visible
    ({"WORLD_SIZE": "4", "LOCAL_WORLD_SIZE": "4", "LOCAL_RANK": "2"}, 8, 5, [2]),  # rank, not current device
    ({"WORLD_SIZE": "4"}, 8, 5, [5]),                                 # no local info: current device
    ({"OMPI_COMM_WORLD_LOCAL_SIZE": "4", "OMPI_COMM_WORLD_LOCAL_RANK": "1"}, 8, 0, [1]),  # MPI launcher
    ({"OMPI_COMM_WORLD_LOCAL_SIZE": "1", "WORLD_SIZE": "4"}, 4, 0, [0, 1, 2, 3]),
    ({"LFM_GPUS": "0,0,1", "WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8"}, 2, 0, [0, 0, 1]),  # explicit list wins
    ({"LFM_GPUS": "3"}, 8, 0, [0, 1, 2]),
    ({}, 0, -1, []),                                                  # no device
])
def test_default_device_policy(lfmlib, monkeypatch, env, nvis, current, want):
    """The writers' default device list (lfm_default_devices, the policy
    behind writeImage / writeKLBstack on a node): the number of processes on
    the node decides, and a rank maps to LOCAL_RANK modulo the visible devices."""
    for v in _LAUNCH_VARS:
        monkeypatch.delenv(v, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert lfmlib.default_devices(nvis, current) == want


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_gpus_flag_is_authoritative():
    """bench.py --gpus N: with no WORLD_SIZE and N > 1 it launches N ranks
    (torchrun child, 127.0.0.1 rendezvous); under a launcher WORLD_SIZE must
    equal N; nccl needs N visible devices."""
    b = _bench()
    assert b.rank_layout(1, {}, 1) == (1, 0, 0, 1)
    assert b.rank_layout(8, {}, 8) == (None, 0, 0, 8)
    assert isinstance(b.rank_layout(8, {}, 1), str)
    assert b.rank_layout(2, {"LFM_BENCH_BACKEND": "gloo"}, 1) == (None, 0, 0, 2)
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2", "LOCAL_WORLD_SIZE": "4"}
    assert b.rank_layout(4, env, 4) == (4, 2, 2, 4)
    assert isinstance(b.rank_layout(8, env, 8), str)
    assert isinstance(b.rank_layout(1, env, 8), str)
    cmd = b.torchrun_cmd(4, ["--gpus", "4", "--steps", "3"], 29512)
    assert cmd[cmd.index("-m") + 1] == "torch.distributed.run"
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_refuses_world_size_mismatch():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero before any
    device call (runs on the CPU)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in r.stderr
