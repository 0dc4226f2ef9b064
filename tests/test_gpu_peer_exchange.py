"""The peer exchange (fmidx.sharding.PeerExchange, SURVEY §8e / BASELINE
configs[3]) across PROCESSES: two ranks, each its own process with its own
doc-range shard (halo 32), swap their payload buffers' IPC handles
(fm_ipc_handle / fm_ipc_open) and OR each other's payloads in place
(fm_shard_or_rows_peers).  On the one-GPU box both ranks share the GPU, so
the group is gloo and the barrier is the host one or the flag words (no
collective per step at all: each rank's signal kernel stores the step number
into the other's flag array, its OR pass waits for them); RCCL refuses two
ranks on one device, so the stream-ordered RCCL barrier runs in the world-1
test of test_gpu_shard_processors.py and in bench.py at N > 1.  Each rank checks,
bit for bit, against the unsharded index it builds too:
  * ShardedDecoder(reduce="peer") over 14 steps with restarts, a step where
    every row restarts (every payload a bitmap) and the double-buffered
    payloads rewritten many times;
  * the Seq processor over ShardedIndex(exchange="peer")."""
import os
import socket
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD, HALO, V = 2, 32, 128256


def _corpus():
    rng = np.random.default_rng(17)
    docs = [rng.integers(0, 900, size=int(rng.integers(5, 300))).tolist() for _ in range(400)]
    for d in docs[::4]:
        d[:4] = [1, 2, 3, 4]
    return docs


def _child(rank, world, port, outdir, barrier):
    import torch
    import torch.distributed as dist

    import fmidx.processors as P
    from fmidx.index import FMIndex
    from fmidx.sharding import ShardedDecoder, ShardedIndex, shard_corpus

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world, rank=rank)
    try:
        docs = _corpus()
        full = FMIndex()
        full.initialize(docs, in_memory=True)
        sd, _ = shard_corpus(docs, world, rank, HALO)
        ix = FMIndex()
        ix.initialize(sd, in_memory=True)
        F = [t for d in reversed(docs) for t in d]
        rng = np.random.default_rng(5)          # the same rows on both ranks
        B = 48
        starts = rng.integers(0, len(F) - 40, size=B)
        pats = [F[a:a + 2] for a in starts]
        dec = ShardedDecoder(ix, V, 10, group=dist.group.WORLD, reduce="peer", halo=HALO, peer_barrier=barrier)
        ref = ShardedDecoder(full, V, 10)
        dec.start(pats, "cuda")
        ref.start(pats, "cuda")
        bad = []
        for step in range(14):
            tok = [F[a + 2 + step] if rng.random() < 0.85 else int(rng.integers(-1, 900)) for a in starts]
            if step == 7:
                tok = [-1] * B                  # every row restarts: wide on both shards
            t = torch.tensor(tok, dtype=torch.int64, device="cuda")
            got = dec.step(t)
            want = ref.step(t)
            if not torch.equal(got, want):
                bad.append(f"decoder step {step}")
        assert dec._peer.step == 14
        if barrier == "flags" and dec._peer.errors():
            bad.append(f"flag barrier timed out at step {dec._peer.errors()}")
        dec.close()
        mk = lambda index: P.SeqIndexBasedLogitsProcessor(index=index, num_beams=1)  # noqa: E731
        pr_ref = mk(full)
        sidx = ShardedIndex(ix, full.occurring_distinct, group=dist.group.WORLD, halo=HALO, exchange="peer",
                            peer_barrier=barrier)
        pr = mk(sidx)
        for step in range(5):
            ids = torch.tensor([[1] + F[a:a + 1 + step] for a in starts[:16]], dtype=torch.int64).cuda()
            scores = torch.from_numpy(rng.standard_normal((16, V)).astype(np.float32)).cuda()
            if not torch.equal(pr(ids, scores.clone()).view(torch.int32), pr_ref(ids, scores.clone()).view(torch.int32)):
                bad.append(f"processor step {step}")
        sidx.close()
        with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
            f.write("\n".join(bad) if bad else "ok")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("barrier", ["host", "flags"])
def test_peer_exchange_two_processes(tmp_path, barrier):
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.spawn(_child, args=(WORLD, port, str(tmp_path), barrier), nprocs=WORLD, join=False)
    deadline = time.time() + 240
    try:
        while not ctx.join(timeout=5):
            if time.time() > deadline:
                pytest.fail("peer-exchange ranks did not finish in 240 s")
    finally:
        for p in ctx.processes:
            if p.is_alive():
                p.kill()
    for r in range(WORLD):
        assert (tmp_path / f"r{r}.txt").read_text() == "ok", r
