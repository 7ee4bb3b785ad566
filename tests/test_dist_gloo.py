"""world_size-2 gloo tests of the multi-process decomposition (knn_dist.py)
on CPU, with the oracle as the per-rank compute: the N>1 paths of bench.py
and of the train-sharded mode, without a GPU."""
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=3000, m=257, d=24, classes=5, seed=4):
    rng = np.random.default_rng(seed)
    centres = rng.uniform(-2, 2, (classes, d))
    lab = rng.integers(0, classes, n + m).astype(np.int32)
    X = np.round((centres[lab] + rng.standard_normal((n + m, d))) * 1024) / 1024
    return X[:n].copy(), lab[:n].copy(), X[n:].copy()


def _tie_data(n=2500, m=120, d=12, classes=5, seed=71):
    """Integer codes 0..255 around 5 centres: many exactly equal distances
    (the reference's own kind of data: MNIST pixels are integers)."""
    rng = np.random.default_rng(seed)
    centres = rng.integers(0, 256, (classes, d))
    lab = rng.integers(0, classes, n + m).astype(np.int32)
    X = np.clip(centres[lab] + rng.integers(-5, 6, (n + m, d)), 0, 255).astype(np.float64)
    return X[:n].copy(), lab[:n].copy(), X[n:].copy()


def _worker(rank, world, port, mode, out_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    import dist_ref
    kd = _load("knn_dist", os.path.join(ROOT, "-mpi-knn-_amd", "knn_dist.py"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr, lab, te = _data()
    n, m, k = tr.shape[0], te.shape[0], 7
    if mode == "normalize":
        # each rank its row shard of train / test (≙ batch_train / batch_test)
        va = te[::3].copy()
        shards = []
        for a in (tr, te, va):
            r0, r1 = kd.shard_range(a.shape[0], world, rank)
            shards.append(torch.from_numpy(a[r0:r1].copy()))
        mx, mn = kd.normalize_sharded(shards, dist_ref.minmax_fold, dist_ref.minmax_apply,
                                      tr.shape[1])
        full = [kd.gather_slices(s, a.shape[0]).numpy() for s, a in zip(shards, (tr, te, va))]
        result = dict(tr=full[0], te=full[1], va=full[2], mx=mx.numpy(), mn=mn.numpy())
    elif mode == "query":
        X = torch.from_numpy(tr) if rank == 0 else torch.zeros_like(torch.from_numpy(tr))
        L = torch.from_numpy(lab) if rank == 0 else torch.zeros(n, dtype=torch.int32)
        kd.broadcast_train(X, L)                       # ≙ MPI_Bcast cpp:224-225
        q0, q1 = kd.shard_range(m, world, rank)        # ≙ MPI_Scatter cpp:226
        got, _, _ = oracle.knn(X.numpy(), L.numpy(), te[q0:q1], k, True, 5, nthreads=2)
        full = kd.gather_slices(torch.from_numpy(got), m)  # ≙ MPI_Gather cpp:383
        el = kd.timed(lambda: None, 3, 1, lambda: None)
        result = dict(labels=full.numpy(), el=np.array([el]))
    elif mode == "train_ties":
        # integer data full of exact distance ties, 3 shards of unequal size:
        # the flagged queries take every shard's distances to their owner,
        # which sorts them as the reference's std::sort does
        tr, lab, te = _tie_data()
        n, m, k = tr.shape[0], te.shape[0], 10
        w = k + 1
        r0, r1 = kd.shard_range(n, world, rank)
        q0, q1 = kd.shard_range(m, world, rank)
        slice_out = {}

        def search_partial(Q):
            return tuple(torch.from_numpy(a) for a in
                         dist_ref.sorted_partial(tr[r0:r1], r0, lab[r0:r1], Q, w))

        def merge_vote(gd, gi, gl, parts, a, b):
            pend = []
            labs, idx, _ = dist_ref.merge_vote(gd.numpy(), gi.numpy(), gl.numpy(), k, a, b, pend)
            slice_out.update(labs=labs, idx=idx, pend=np.array(pend, np.int64))
            return torch.from_numpy(labs)

        class Ties:
            n_total = n

            def pending(self):
                return torch.from_numpy(slice_out["pend"])

            def shard_distances(self, sel):
                return torch.from_numpy(np.stack([oracle.row_distances(te[int(q)], tr[r0:r1])
                                                  for q in sel.numpy()]))

            def resolve(self, D, rows, orow):
                T, off = orow.numel(), np.cumsum([0] + list(rows))
                Dn = D.numpy()
                for i, o in enumerate(orow.numpy()):
                    Dq = np.concatenate([Dn[T * off[g] + i * rows[g]:T * off[g] + (i + 1) * rows[g]]
                                         for g in range(len(rows))])
                    lb, ix = oracle.sort_vote(Dq, lab, k, 5, n_out=k)
                    slice_out["labs"][o], slice_out["idx"][o] = lb, ix

        kd.train_sharded(search_partial, merge_vote, te, m, w, k, ties=Ties())
        labs = kd.gather_slices(torch.from_numpy(slice_out["labs"]), m)
        idx = kd.gather_slices(torch.from_numpy(slice_out["idx"]), m)
        npend = torch.tensor([len(slice_out["pend"])])
        dist.all_reduce(npend)
        result = dict(labels=labs.numpy(), idx=idx.numpy(), pending=npend.numpy())
    else:
        if mode == "train_bigk":
            # any K <= N_train like cpp:328: the union of the ranks' lists
            # (2 x 3001) is beyond the LDS merge's 4096 entries
            tr, lab, te = _data(n=8000, m=24, d=12)
            n, m, k = tr.shape[0], te.shape[0], 3000
        w = k + 1
        r0, r1 = kd.shard_range(n, world, rank)

        def search_partial(Q):
            _, idx, dd = oracle.knn(tr[r0:r1], lab[r0:r1], Q, w, True, 5, n_out=w, nthreads=2)
            gl = lab[r0:r1][idx]
            return (torch.from_numpy(dd), torch.from_numpy(idx + r0), torch.from_numpy(gl))

        def merge_vote(gd, gi, gl, parts, q0, q1):
            labs, _, _ = dist_ref.merge_vote(gd.numpy(), gi.numpy(), gl.numpy(), k, q0, q1)
            return torch.from_numpy(labs)

        mine, (q0, q1) = kd.train_sharded(search_partial, merge_vote, te, m, w, k)
        full = kd.gather_slices(mine, m)
        result = dict(labels=full.numpy())
    if rank == 0:
        np.savez(out_path, **result)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_normalisation_matches_oracle(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    out = str(tmp_path / "n.npz")
    mp.spawn(_worker, args=(2, _free_port(), "normalize", out), nprocs=2, join=True)
    tr, _, te = _data()
    va = te[::3].copy()
    oracle.normalize(tr, te, va)
    got = np.load(out)
    for name, want in (("tr", tr), ("te", te), ("va", va)):
        assert got[name].tobytes() == want.tobytes(), name


@pytest.mark.parametrize("mode", ["query", "train", "train_bigk"])
def test_two_rank_decomposition_matches_single_process(mode, tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True)
    if mode == "train_bigk":
        tr, lab, te = _data(n=8000, m=24, d=12)
        want, _, _ = oracle.knn(tr, lab, te, 3000, True, 5)
    else:
        tr, lab, te = _data()
        want, _, _ = oracle.knn(tr, lab, te, 7, True, 5)
    got = np.load(out)["labels"]
    np.testing.assert_array_equal(got, want)


def test_three_rank_reference_tie_order(tmp_path):
    """Train-sharded mode on tie-heavy integer data over 3 gloo ranks
    (ragged shards): the merge flags every query with an exact tie in its
    top k, the flagged queries' distances to every shard go to their owner
    (all-gather of ids + all-to-all of distance blocks, knn_dist.resolve_ties)
    and the owner's std::sort over the whole train set gives the reference's
    labels AND neighbour order for every query."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    out = str(tmp_path / "t.npz")
    mp.spawn(_worker, args=(3, _free_port(), "train_ties", out), nprocs=3, join=True)
    tr, lab, te = _tie_data()
    want, widx, _ = oracle.knn(tr, lab, te, 10, True, 5, n_out=10)
    got = np.load(out)
    assert int(got["pending"][0]) > 30, "expected many tied queries"
    np.testing.assert_array_equal(got["labels"], want)
    np.testing.assert_array_equal(got["idx"], widx)


def test_shard_ranges_cover_ragged():
    kd = _load("knn_dist", os.path.join(ROOT, "-mpi-knn-_amd", "knn_dist.py"))
    for n in (0, 1, 7, 10000, 10001):
        for world in (1, 2, 3, 8):
            spans = [kd.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def _bench_line(args):
    import json
    import subprocess
    import sys
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_bench_launches_its_own_ranks():
    """bench.py --gpus 2 starts two ranks itself (torch.distributed.run as a
    child, gloo in --dry-run): the line reports n_gpus 2 and the gathered
    labels equal the one-rank run of the same total query set."""
    common = ["--dry-run", "--n-train", "3000", "--dim", "24", "--steps", "2", "--warmup", "1"]
    one = _bench_line(common + ["--gpus", "1", "--queries", "96"])
    two = _bench_line(common + ["--gpus", "2", "--queries", "48"])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["dry_run"] and two["value"] is None
    assert two["labels_sha1"] == one["labels_sha1"]
    # the N>1 line's extra legs are wired: the native drop-in through
    # knn_group in both modes (commands only on CPU) and the train-sharded
    # decomposition (labels equal the query-sharded run's)
    assert "--gpus 2 --mode query" in two["group_query"]["cmd"]
    assert "--gpus 2 --mode train" in two["group_train"]["cmd"]
    assert "--Normalize true" in two["group_train"]["cmd"]
    assert two["group_query"]["value"] is None and two["train_sharded"]["value"] is None
    assert sorted(two["dropin_inputs"]) == ["mnist_test.csv", "mnist_train.csv",
                                            "mnist_validation.csv"]
    assert two["train_sharded"]["labels_match"] and one["train_sharded"]["labels_match"]
    # the N-GPU line's self-checks: one entry per rank for the candidate
    # kernel time, rescans and tie counts (main leg) and the tie resolutions
    # (train-sharded leg); rank 0's label sha1 equals the 1-rank run over the
    # same query rows; the train-sharded labels' sha1 is the same at every N
    one48 = _bench_line(common + ["--gpus", "1", "--queries", "48"])
    for key in ("kernel_ms", "rescanned_queries", "tie_vote_queries", "tie_reordered_queries",
                "labels_sha1"):
        assert len(two["per_rank"][key]) == 2 and len(one48["per_rank"][key]) == 1, key
    assert two["per_rank"]["labels_sha1"][0] == one48["per_rank"]["labels_sha1"][0]
    assert two["labels_sha1_rank0"] == one48["labels_sha1_rank0"]
    assert two["per_rank"]["labels_sha1"][1] != two["per_rank"]["labels_sha1"][0]
    for key in ("kernel_ms", "tie_resolved_queries", "tie_pending_queries"):
        assert len(two["train_sharded"]["per_rank"][key]) == 2, key
    assert two["train_sharded"]["labels_sha1"] == one48["train_sharded"]["labels_sha1"]


def test_bench_failure_names_rank_and_phase():
    """A failing rank exits non-zero and names itself and the phase it was in
    (a negative --n-train makes the dry run's data generation fail)."""
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--n-train",
                          "-5", "--dim", "24", "--queries", "8", "--steps", "1", "--warmup", "0"],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode != 0
    assert "rank 0 of 1 FAILED in phase" in out.stderr, out.stderr[-1500:]
