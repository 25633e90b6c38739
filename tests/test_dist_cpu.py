"""World-size-2 gloo test of the sharded search-round protocol (SearchEngine):
candidates sharded by global index, one all_gather of scores per round, identical
argmax on every rank and equal to the single-process result. The sampler/verifier
are CPU stand-ins here (the GPU path is covered by tests/test_gpu_parity.py)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from itsd.search import SearchEngine


class _Model:
    device = torch.device("cpu")


class _Sampler:
    model = _Model()

    def run(self, x, labels=None, seed=0, noise_offset=0, graph=True):
        x.copy_(torch.tanh(x * 1.3))
        return x


class _Verifier:
    kind = 0

    def score_batch(self, images, n_cand):
        v = images.reshape(n_cand, -1).double()
        return 1.0 / (1.0 + v.var(dim=1))


class CPUEngine(SearchEngine):
    def candidate_noise(self, round_id, g0, count, shape, pivot=None, scale=1.0):
        outs = []
        for g in range(g0, g0 + count):
            gen = torch.Generator().manual_seed(self.seed * 1_000_003 + round_id * 10_007 + g)
            z = torch.randn(shape, generator=gen)
            outs.append(z * scale + (pivot if pivot is not None else 0))
        return torch.cat(outs)


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = CPUEngine(_Sampler(), _Verifier(), seed=3)
    noise, score, info = eng.random_search(8, (1, 3, 4, 4))
    rs_image = eng.best_image.clone()
    zo_noise, zo_score, hist = eng.zero_order_search(torch.zeros(1, 3, 4, 4), 6, 0.95, 3)
    torch.save({"rank": rank, "score": score, "best": info["best_index"], "noise": noise, "scores": info["scores"],
                "zo_score": zo_score, "zo_noise": zo_noise, "zo_hist": hist["best_index"],
                "rs_image": rs_image, "zo_image": eng.best_image.clone()},
               f"{out_path}.{rank}")
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_rounds_agree_with_single_process():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res")
        mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        r0 = torch.load(out + ".0", weights_only=False)
        r1 = torch.load(out + ".1", weights_only=False)
    single = CPUEngine(_Sampler(), _Verifier(), seed=3)
    noise, score, info = single.random_search(8, (1, 3, 4, 4))
    rs_image = single.best_image.clone()
    zo_noise, zo_score, hist = single.zero_order_search(torch.zeros(1, 3, 4, 4), 6, 0.95, 3)
    # the winner's image (kept by its owner, broadcast at the end) is the one that was scored
    assert torch.equal(rs_image, torch.tanh(noise * 1.3))
    assert abs(_Verifier().score_batch(rs_image, 1).item() - score) < 1e-12
    for r in (r0, r1):
        assert torch.equal(r["rs_image"], rs_image) and torch.equal(r["zo_image"], single.best_image)
        assert r["best"] == info["best_index"] and r["score"] == score
        assert r["scores"] == info["scores"]
        assert torch.equal(r["noise"], noise)
        assert r["zo_score"] == zo_score and r["zo_hist"] == hist["best_index"]
        assert torch.equal(r["zo_noise"], zo_noise)


def test_nan_scores_never_win_and_all_nan_round():
    """search_algorithm.py:79: `score > best_score` from -inf -- NaN never wins, ties go to
    the lowest index, and a round of only NaN scores keeps the reference's initial best."""
    from itsd.search import strict_argmax

    nan = float("nan")
    assert strict_argmax(torch.tensor([0.1, nan, 0.3, 0.3], dtype=torch.float64)) == (2, 0.3)
    assert strict_argmax(torch.tensor([nan, nan])) == (-1, float("-inf"))

    class NaNVerifier(_Verifier):
        def score_batch(self, images, n_cand):
            return torch.full((n_cand,), nan, dtype=torch.float64)

    eng = CPUEngine(_Sampler(), NaNVerifier(), seed=0)
    best, score, info = eng.random_search(4, (1, 3, 4, 4))
    assert best is None and score == float("-inf") and info["best_index"] == -1  # (None, -inf)
    init = torch.ones(1, 3, 4, 4)
    zb, zs, _ = eng.zero_order_search(init, 3, 0.95, 2)
    assert torch.equal(zb, init) and zs == float("-inf")
    pb, ps, _ = eng.path_search(init, 3, 0.1)
    assert torch.equal(pb, init) and ps == float("-inf")


def test_uneven_shard_rejected():
    eng = CPUEngine(_Sampler(), _Verifier(), seed=0)
    eng.world, eng.rank = 3, 0
    with pytest.raises(ValueError):
        eng.shard(8)
