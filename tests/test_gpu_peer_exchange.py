"""The peer exchange (fmidx.sharding.PeerExchange, SURVEY §8e / BASELINE
configs[3]) across PROCESSES: two ranks, each its own process with its own
doc-range shard (halo 32), swap their payload buffers' IPC handles
(fm_ipc_handle / fm_ipc_open) and OR each other's payloads in place
(fm_shard_or_rows_peers).  On the one-GPU box both ranks share the GPU, so
the group is gloo and the barrier is the host one or the flag words (no
collective per step at all: each rank's signal kernel advances its device
step counter and stores it into the other's flag array, its OR pass waits for
them); RCCL refuses two ranks on one device, so the stream-ordered RCCL
barrier runs in the world-1 test of test_gpu_shard_processors.py and in
bench.py at N > 1.  Each rank checks, bit for bit, against the unsharded index
it builds too:
  * ShardedDecoder(reduce="peer") over 14 steps with restarts, a step where
    every row restarts (every payload a bitmap) and the double-buffered
    payloads rewritten many times; with the flag barrier also as ONE captured
    step graph replayed for every step (graph=True);
  * the Seq processor over ShardedIndex(exchange="peer");
  * the Qwen processor over the default ShardedIndex (peer + flags) where the
    device path hands over to the host path: a row without the end marker,
    and boosts BOOST * 2^k past the float range (bf16: inf written, as the
    reference writes it; fp32: the reference's RuntimeError raised);
and, separately, the flag barrier's timeout: rank 1 skips its signal for one
step, and both ranks raise PeerBarrierTimeout at that step instead of
returning its mask (check="deferred": at the next call)."""
import os
import socket
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD, HALO, V = 2, 32, 128256
MARKER = [151645, 198, 151644, 77091, 198]
THINK = [151667, 271, 151668, 271]


def _corpus():
    rng = np.random.default_rng(17)
    docs = [rng.integers(0, 900, size=int(rng.integers(5, 300))).tolist() for _ in range(400)]
    for d in docs[::4]:
        d[:4] = [1, 2, 3, 4]
    for d in docs[::7]:
        d[-1] = 2                        # eos occurs in the corpus (count([eos]) > 0)
    return docs


def _outcome(fn):
    """('ok', int view of the output) or (exception type name, message)."""
    import torch

    try:
        out = fn()
    except Exception as e:  # noqa: BLE001 -- the reference's exception is the expected outcome
        return type(e).__name__, str(e)
    return "ok", out.view(torch.int32 if out.dtype == torch.float32 else torch.int16).cpu()


def _same(a, b):
    import torch

    if a[0] != b[0]:
        return False
    return torch.equal(a[1], b[1]) if a[0] == "ok" else a[1] == b[1]


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
        bad = []
        for graph in ([False, True] if barrier == "flags" else [False]):
            dec = ShardedDecoder(ix, V, 10, group=dist.group.WORLD, reduce="peer", halo=HALO, peer_barrier=barrier,
                                 graph=graph)
            ref = ShardedDecoder(full, V, 10)
            dec.start(pats, "cuda")
            ref.start(pats, "cuda")
            srng = np.random.default_rng(9)
            for step in range(14):
                tok = [F[a + 2 + step] if srng.random() < 0.85 else int(srng.integers(-1, 900)) for a in starts]
                if step == 7:
                    tok = [-1] * B                  # every row restarts: wide on both shards
                t = torch.tensor(tok, dtype=torch.int64, device="cuda")
                got = dec.step(t)
                want = ref.step(t)
                if not torch.equal(got, want):
                    bad.append(f"decoder step {step} (graph {graph})")
            if dec._peer.step != 14:
                bad.append(f"{dec._peer.step} exchange steps (graph {graph})")
            if barrier == "flags" and dec._peer.errors():
                bad.append(f"flag barrier timed out at step {dec._peer.errors()} (graph {graph})")
            if graph and dec._g is None:
                bad.append("graph mode captured no step")
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
        if barrier == "flags":
            bad += _qwen_host_path_cases(full, ix, F, rng)
        with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
            f.write("\n".join(bad) if bad else "ok")
    finally:
        dist.destroy_process_group()


def _qwen_host_path_cases(full, ix, F, rng):
    """Inputs the Qwen device path hands to the host path, over the default
    ShardedIndex (peer exchange, flag barrier): the sharded processor's outcome
    == the unsharded one's (output bit for bit, or the same exception)."""
    import torch
    import torch.distributed as dist

    import fmidx.processors as P
    from fmidx.sharding import ShardedIndex

    bad = []
    # the processors' default exchange over gloo is "sparse" (auto: peer needs an RCCL group on one
    # host); the peer exchange with the flag barrier is asked for explicitly here
    assert ShardedIndex(ix, full.occurring_distinct, group=dist.group.WORLD, halo=HALO).exchange == "sparse"
    sidx = ShardedIndex(ix, full.occurring_distinct, group=dist.group.WORLD, halo=HALO, exchange="peer")
    assert sidx.exchange == "peer" and sidx.peer_barrier == "flags"
    kw = dict(num_beams=1, min_new_tokens=3, always_allow_eos=True, length_reward_factor=2.0)
    ref_p = P.QwenIndexBasedLogitsProcessor(index=full, **kw)
    sh_p = P.QwenIndexBasedLogitsProcessor(index=sidx, **kw)
    B = 8
    starts = rng.integers(0, len(F) - 200, size=B)
    prompt = [100, 101] + MARKER

    def rows(k):
        out = []
        for b in range(B):
            s = list(F[int(starts[b]):int(starts[b]) + 6])
            if b % 4 == 1:
                s = [int(x) for x in rng.integers(0, 900, size=k - 1)] + [2]   # k tokens ending in eos
                out.append(prompt + THINK + s)
            elif b % 4 == 2:
                out.append(prompt + s)                                          # never finished thinking
            else:
                out.append(prompt + THINK + s)
        width = max(len(r) for r in out)
        return [r + [0] * (width - len(r)) if len(r) < width else r for r in out]

    cases = []
    # (a) boosts 10 * 2^k past the float range: bf16 writes inf (device path), fp32 raises as the reference
    r = rows(130)
    cases += [("k>=125 bf16", r, torch.bfloat16), ("k>=125 fp32", r, torch.float32)]
    # (b) a row without the end marker (the reference's remove_end_marker drops it): the host path
    r2 = rows(8)
    r2[3] = [100, 101, 102, 103, 104, 105, 106] + r2[3][7:]
    cases += [("no marker bf16", r2, torch.bfloat16), ("no marker fp32", r2, torch.float32)]
    # (c) an ordinary call after them: the sharded state keeps working
    cases += [("ordinary", rows(6), torch.bfloat16)]
    for name, ids_l, dt in cases:
        ids = torch.tensor(ids_l, dtype=torch.int64).cuda()
        scores = torch.from_numpy(rng.standard_normal((B, V)).astype(np.float32)).to(dt).cuda()
        want = _outcome(lambda: ref_p(ids, scores.clone()))
        got = _outcome(lambda: sh_p(ids, scores.clone()))
        if not _same(want, got):
            bad.append(f"qwen {name}: sharded {got[0]} vs unsharded {want[0]} "
                       f"{got[1] if got[0] != 'ok' else ''} / {want[1] if want[0] != 'ok' else ''}")
        if name == "k>=125 bf16" and want[0] == "ok":
            x = ref_p(ids, scores.clone()).float()
            if not torch.isinf(x).any():
                bad.append("k>=125 bf16: no inf boost in the reference output")
        if name == "k>=125 fp32" and want[0] != "RuntimeError":
            bad.append(f"k>=125 fp32: the unsharded processor gave {want[0]}, expected the reference's RuntimeError")
    sidx.close()
    return bad


@pytest.mark.parametrize("barrier", ["host", "flags"])
def test_peer_exchange_two_processes(tmp_path, barrier):
    _spawn(_child, tmp_path, barrier, 240)


def _timeout_child(rank, world, port, outdir, _):
    """Rank 1 skips its flag-barrier signal at step 3: the step's OR pass times
    out on both ranks (spin bound 2^16 polls, tens of ms).  With the default
    check="sync" both ranks raise PeerBarrierTimeout AT step 3 -- the step that
    timed out returns no mask (exact or absent); with the opt-in
    check="deferred" the raise comes at the next call (step 4), as documented.
    close() raises it too, either way."""
    import torch
    import torch.distributed as dist

    from fmidx.index import FMIndex
    from fmidx.sharding import PeerBarrierTimeout, ShardedDecoder, shard_corpus

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world, rank=rank)
    try:
        docs = _corpus()
        sd, _ = shard_corpus(docs, world, rank, HALO)
        ix = FMIndex()
        ix.initialize(sd, in_memory=True)
        F = [t for d in reversed(docs) for t in d]
        rng = np.random.default_rng(5)
        B = 32
        starts = rng.integers(0, len(F) - 40, size=B)
        res = []
        for check, want_at in (("sync", 3), ("deferred", 4)):
            dec = ShardedDecoder(ix, V, 10, group=dist.group.WORLD, reduce="peer", halo=HALO, peer_barrier="flags",
                                 spins=1 << 16, check=check)
            dec.start([F[a:a + 2] for a in starts], "cuda")
            raised_at, msgs, returned = None, [], []
            for step in range(6):
                dist.barrier()                  # the ranks start each step together: only the skip times out
                if step == 3 and rank == 1:
                    dec._peer._skip_signal = 1
                t = torch.tensor([F[a + 2 + step] for a in starts], dtype=torch.int64, device="cuda")
                try:
                    dec.step(t)
                    returned.append(step)
                except PeerBarrierTimeout as e:
                    raised_at = step
                    msgs.append(str(e))
                    break
                torch.cuda.synchronize()        # deferred: the pass (and its error word) done before the next call
            closed_raises = False
            try:
                dec.close()
            except PeerBarrierTimeout:
                closed_raises = True
            # the device step counter is 1-based: host step s is exchange step s + 1
            if not (raised_at == want_at and closed_raises and bool(msgs) and "step 4" in msgs[0] and
                    (check == "deferred" or 3 not in returned)):
                res.append(f"{check}: raised at {raised_at} (want {want_at}), close raised {closed_raises}, "
                           f"returned {returned}, {msgs}")
        with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
            f.write("\n".join(res) if res else "ok")
    finally:
        dist.destroy_process_group()


def test_flag_barrier_timeout_raises(tmp_path):
    _spawn(_timeout_child, tmp_path, None, 180)


def _spawn(fn, tmp_path, arg, limit):
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.spawn(fn, args=(WORLD, port, str(tmp_path), arg), nprocs=WORLD, join=False)
    deadline = time.time() + limit
    try:
        while not ctx.join(timeout=5):
            if time.time() > deadline:
                pytest.fail(f"ranks did not finish in {limit} s")
    finally:
        for p in ctx.processes:
            if p.is_alive():
                p.kill()
    for r in range(WORLD):
        assert (tmp_path / f"r{r}.txt").read_text() == "ok", (r, (tmp_path / f"r{r}.txt").read_text())


def test_bench_peer_preflight_two_processes(tmp_path):
    """bench.py --peer-preflight, the child each rank runs before the N > 1 sharded leg's peer
    modes: two children (RANK 0 / 1 of WORLD_SIZE 2) on this box's one GPU
    (FMIDX_PREFLIGHT_DEVICE=0) map each other's buffers, decode 6 steps with the flag barrier
    and check="sync", and both exit 0 (exact against the unsharded index)."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), FMIDX_PREFLIGHT_DEVICE="0",
                   FMIDX_PREFLIGHT_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(repo, "bench.py"), "--peer-preflight"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=200)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert [p.returncode for p in procs] == [0, 0], outs
