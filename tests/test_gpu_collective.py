"""The replay path's only collective on real hardware: per-document checksums
written by the device straight into a torch tensor (mt_checksums_device) and all-gathered
over RCCL (torch.distributed backend "nccl") by the same code bench.py runs after its timed
region (shard.gather_checksums, bench.verify_shards).  One GPU, so a world-1 process group:
the collective, the device-side fill and the padding/trim logic all execute; the N > 1
rank arithmetic is covered over gloo by tests/test_multirank.py."""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture()
def nccl_world1():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_gpu_rccl_checksum_allgather_equals_host_checksums(nccl_world1, oracle_lib):
    import torch
    import bench
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.shard import gather_checksums
    from fluidframework_amd.wire import CHECKSUM_DTYPE
    dist = nccl_world1
    assert dist.get_backend() == "nccl"
    cfg = dict(json.load(open(os.path.join(REPO, "bench", "configs.json")))["c3"], ops=600)
    docs, base = 37, 0                          # odd count: no power-of-two padding luck
    mt = MergeTreeBatch(docs, device=0, **bench.capacities(cfg))
    batch = mt.generate(cfg, base)
    gen = mt.checksums()
    seed_off, seed = mt.generated_seeds(cfg, base)
    mt.load_initial_text(seed_off, seed)
    mt.reset()
    batch.apply_async()
    mt.sync()
    host = mt.checksums()
    assert (mt.status() == 0).all()
    local = torch.full((docs * CHECKSUM_DTYPE.itemsize,), 0xAB, dtype=torch.uint8, device="cuda")
    mt.checksums_device(local.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(local.cpu().numpy().view(CHECKSUM_DTYPE), host)
    got = gather_checksums(local, dist, device=torch.device("cuda", 0), n_total=docs)
    assert got.tobytes() == host.tobytes() == gen.tobytes()
    # bench.py's exchange step itself: replay == generation, and sampled documents equal
    # the CPU oracle's replay of the same global documents
    rep = bench.verify_shards(dist, 0, 1, docs, dict(cfg), local, gen, torch.device("cuda", 0), 3, 2)
    assert rep["docs_gathered"] == docs and rep["replay_equals_generation"]
    assert rep["oracle_docs"] == 3 and rep["oracle_mismatches"] == 0
