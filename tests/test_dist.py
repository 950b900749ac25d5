"""Multi-rank exchange on CPU (gloo, world_size 2): the collective layer of the
multi-GPU path (kmerjs_amd/multi.py) without a GPU.  The device reduce that
consumes the gathered partials is covered by the GPU sharded-merge tests."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kmerjs_amd import multi


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeCounter:
    """Stands in for Counter's record export/import (host-side record keys)."""

    def __init__(self, recs):
        self.recs = dict(recs)

    def records_export(self):
        items = sorted(self.recs.items(), key=lambda kv: kv[1][1])
        kb = b"".join(k for k, _ in items)
        off = np.cumsum([0] + [len(k) for k, _ in items]).astype(np.uint64)
        return kb, off, np.array([v[0] for _, v in items], dtype=np.uint64), \
            np.array([v[1] for _, v in items], dtype=np.uint64)

    def records_clear(self):
        self.recs = {}

    def records_import(self, kb, off, cnt, fst):
        for i in range(len(cnt)):
            key = kb[int(off[i]):int(off[i + 1])]
            c, f = self.recs.get(key, (0, 1 << 63))
            self.recs[key] = (c + int(cnt[i]), min(f, int(fst[i])))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = [5, 0, 3][rank]
        keys = torch.arange(n, dtype=torch.int64) + 100 * rank
        vals = torch.stack([keys * 10, torch.ones(n, dtype=torch.int64)], dim=1) if n else \
            torch.empty((0, 2), dtype=torch.int64)
        gk, gv = multi.gather_partials(keys, vals, pad_key=1 << 22, dst=0)
        ctr = _FakeCounter({b"NNA": (rank + 1, 7 + rank), (b"X%d" % rank): (1, rank)})
        multi.gather_records(ctr, dst=0)
        if rank == 0:
            q.put(("ok", gk.tolist(), gv.tolist(), sorted(ctr.recs.items())))
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_partials_and_records_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, *payload = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", payload
    gk, gv, recs = payload
    sizes = [5, 0, 3][:world]
    maxn = max(sizes)
    assert len(gk) == world * maxn and len(gv) == world * maxn
    for r, n in enumerate(sizes):
        blk = gk[r * maxn:(r + 1) * maxn]
        assert blk[:n] == [100 * r + i for i in range(n)]
        assert all(x == 1 << 22 for x in blk[n:])          # pad key -> dropped by the device reduce
        vb = gv[r * maxn:(r + 1) * maxn]
        assert all(v == [-1, 0] for v in vb[n:])           # pad value: count 0
        assert vb[:n] == [[(100 * r + i) * 10, 1] for i in range(n)]
    recs = dict(recs)
    assert recs[b"NNA"] == (sum(range(1, world + 1)), 7)  # counts add, first = min
    for r in range(world):
        assert recs[b"X%d" % r] == (1, r)


def test_split_at_records_covers_input():
    from oracle import oracle
    data = oracle.synth_fastq(3, 0, 101)
    for world in (1, 2, 3, 8):
        shards = multi.split_at_records(data, world)
        assert b"".join(data[lo:hi] for lo, hi, _ in shards) == data
        for lo, hi, lines_before in shards:
            assert data[:lo].count(b"\n") == lines_before
            assert lines_before % 4 == 0
            assert lo == 0 or data[lo - 1:lo] == b"\n"


def test_shard_plan_positions():
    p = multi.shard_plan(1000, 3)
    assert p == {"first_read": 3000, "lines_before": 12000, "byte_offset": 3000 * 317, "n_reads": 1000}


def test_invalid_key_is_past_every_suffix():
    assert multi.invalid_key(16, 5) == 1 << 22
    assert multi.invalid_key(5, 5) == 1


def _shuffle_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kbits = 22
        g = torch.Generator().manual_seed(rank)
        n = 1000 + 137 * rank
        keys = torch.randint(0, 1 << kbits, (n,), generator=g, dtype=torch.int64)
        # first-occurrence orders of this rank's shard: increasing, above every earlier rank's
        first = torch.arange(n, dtype=torch.int64) + (rank << 40)
        vals = torch.stack([first, torch.full((n,), rank + 1, dtype=torch.int64)], dim=1)
        rk, rv = multi.shuffle_partials(keys, vals, kbits)
        q.put(("ok", rank, keys.tolist(), rk.tolist(), rv.tolist()))
    except Exception as e:  # pragma: no cover
        q.put(("err", rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shuffle_partials_by_key_range_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shuffle_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    by_rank = {r[1]: r for r in res}
    sent = sorted(k for r in res for k in r[2])
    got = []
    for rank in range(world):
        _, _, _, rk, rv = by_rank[rank]
        owners = multi.key_owner(torch.tensor(rk, dtype=torch.int64), 22, world).tolist() if rk else []
        assert all(o == rank for o in owners)                 # only this rank's key range
        firsts = [v[0] for v in rv]
        assert firsts == sorted(firsts)                        # still in first-occurrence order
        got += rk
    assert sorted(got) == sent                                 # nothing lost, nothing duplicated


def _dense_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kbits = 12
        g = torch.Generator().manual_seed(10 + rank)
        n = 700 + 91 * rank
        keys = torch.unique(torch.randint(0, 1 << kbits, (n,), generator=g, dtype=torch.int64))
        keys = keys[torch.randperm(keys.numel(), generator=g)]
        keys = torch.cat([keys, torch.tensor([1 << kbits])])            # + the reduce's invalid sentinel
        first = torch.arange(keys.numel(), dtype=torch.int64) + (rank << 40)
        vals = torch.stack([first, torch.randint(1, 9, (keys.numel(),), generator=g)], dim=1)
        rk, rv = multi.dense_reduce(keys, vals, kbits)
        q.put(("ok", rank, keys.tolist(), vals.tolist(), rk.tolist(), rv.tolist()))
    except Exception as e:  # pragma: no cover
        q.put(("err", rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_dense_reduce_gloo(world):
    """finish_dense's collective (SURVEY §8e dense merge): per key, counts add
    and the first occurrence is the minimum over the ranks; every key lands on
    exactly one rank (its slice of the key space), in first-occurrence order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dense_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    want = {}
    for r in res:
        for key, (f, c) in zip(r[2], r[3]):
            if key < 1 << 12:
                pf, pc = want.get(key, (None, 0))
                want[key] = (f if pf is None else min(pf, f), pc + c)
    got = {}
    per = -(-(1 << 12) // world)
    for r in sorted(res, key=lambda x: x[1]):
        rank, rk, rv = r[1], r[4], r[5]
        assert all(rank * per <= key < (rank + 1) * per for key in rk)
        assert [v[0] for v in rv] == sorted(v[0] for v in rv)
        for key, (f, c) in zip(rk, rv):
            assert key not in got
            got[key] = (f, c)
    assert got == want


def test_key_owner_balanced_and_monotone():
    keys = torch.arange(0, 1 << 22, 97, dtype=torch.int64)
    for world in (1, 2, 3, 8):
        own = multi.key_owner(keys, 22, world)
        assert int(own.min()) == 0 and int(own.max()) == world - 1
        assert bool((own[1:] >= own[:-1]).all())
    big = torch.tensor([(1 << 62) - 1, 0], dtype=torch.int64)
    assert multi.key_owner(big, 62, 8).tolist() == [7, 0]


def _exchange_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # owner-major runs of {order, key} records, as kmer_exchange_prepare lays them out
        counts = [(rank + 1) * (o + 2) % 5 for o in range(world)]
        recs = []
        for o in range(world):
            recs += [[(rank << 40) + 100 * o + i, 1000 * o + i] for i in range(counts[o])]
        send = torch.tensor(recs, dtype=torch.int64).view(-1) if recs else torch.empty(0, dtype=torch.int64)
        recv_counts, rec_counts = multi.exchange_counts(counts, 10 + rank, "cpu")
        recv = multi.exchange_runs(send, counts, recv_counts)
        q.put(("ok", rank, counts, recv_counts, rec_counts, recv.view(-1, 2).tolist()))
    except Exception as e:  # pragma: no cover
        q.put(("err", rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_hit_exchange_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    by_rank = {r[1]: r for r in res}
    for rank in range(world):
        _, _, counts, recv_counts, rec_counts, recv = by_rank[rank]
        assert rec_counts == [10 + r for r in range(world)]          # every rank's record count
        assert recv_counts == [by_rank[src][2][rank] for src in range(world)]
        # run `rank` of every source, concatenated by source rank: global order kept
        want = [[(src << 40) + 100 * rank + i, 1000 * rank + i] for src in range(world)
                for i in range(by_rank[src][2][rank])]
        assert recv == want


def _gather_rows_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # an ordered key range per rank, as collect_ordered_device sends it:
        # n rows of k key bytes, counts, first-occurrence keys
        k, n = 4, [3, 0, 2][rank]
        keys = torch.tensor([[65 + rank, 67, 71, 84 + i % 2] for i in range(n)], dtype=torch.uint8).view(-1) \
            if n else torch.empty(0, dtype=torch.uint8)
        cnt = torch.arange(n, dtype=torch.int64) + 10 * rank
        fst = torch.arange(n, dtype=torch.int64) * world + rank
        got, total = multi.gather_rows([(keys, k), (cnt, 1), (fst, 1)], n, dst=0)
        if rank == 0:
            q.put(("ok", total, got[0].view(-1, k).tolist(), got[1].tolist(), got[2].tolist()))
        else:
            q.put(("ok", total, got, None, None))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rows_alltoallv_gloo(world):
    # the collective of the device-side ordered collect (multi.collect_ordered_device):
    # variable-length row blocks to rank 0 in one alltoallv per tensor, no padding
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    root = [r for r in res if r[1] != 0 or r[2] is not None]
    ns = [[3, 0, 2][r] for r in range(world)]
    main = [r for r in res if r[3] is not None][0]
    _, total, keys, cnt, fst = main
    assert total == sum(ns)
    assert keys == [[65 + r, 67, 71, 84 + i % 2] for r in range(world) for i in range(ns[r])]
    assert cnt == [i + 10 * r for r in range(world) for i in range(ns[r])]
    assert fst == [i * world + r for r in range(world) for i in range(ns[r])]
    assert root


def _table_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # a session's pass-1 keys: h grouped by partition (top 10 bits), as
        # kmer_table_exchange_prepare lays them out (owner-major = partition-major)
        rng = np.random.default_rng(7 + rank)
        h = rng.integers(0, 1 << 63, size=5000 + 1000 * rank, dtype=np.int64) * 2 + rng.integers(0, 2, 1)
        part = (h.view(np.uint64) >> np.uint64(54)).astype(np.int64)
        order = np.argsort(part, kind="stable")
        hs, ps = h[order], part[order]
        parts = np.bincount(ps, minlength=1024)
        counts = [int(parts[slice(*multi.table_part_range(o, world))].sum()) for o in range(world)]
        recv, parts_all = multi.exchange_table_keys(torch.from_numpy(hs), counts, parts.tolist())
        q.put(("ok", rank, recv.numpy().tolist(), parts_all.numpy().tolist()))
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put(("err", rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_table_exchange_collectives_gloo(world):
    """Each rank receives exactly the pass-1 keys of its partitions, source
    rank by source rank, partition-major, and every rank's partition table."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_table_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        status, rank, recv, parts_all = q.get(timeout=120)
        assert status == "ok", recv
        got[rank] = (recv, parts_all)
    for p in procs:
        p.join(timeout=60)
    sent = []
    for r in range(world):
        rng = np.random.default_rng(7 + r)
        h = rng.integers(0, 1 << 63, size=5000 + 1000 * r, dtype=np.int64) * 2 + rng.integers(0, 2, 1)
        part = (h.view(np.uint64) >> np.uint64(54)).astype(np.int64)
        order = np.argsort(part, kind="stable")
        sent.append((h[order], part[order]))
    for o in range(world):
        lo, hi = multi.table_part_range(o, world)
        want = np.concatenate([hs[(ps >= lo) & (ps < hi)] for hs, ps in sent])
        recv, parts_all = got[o]
        assert recv == want.tolist()
        assert parts_all == [np.bincount(ps, minlength=1024).tolist() for _, ps in sent]
    # the owners' ranges tile the 1024 partitions
    assert [multi.table_part_range(o, world)[0] for o in range(world)] + [1024] == \
        [0] + [multi.table_part_range(o, world)[1] for o in range(world)]
