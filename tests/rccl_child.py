"""Child process of tests/test_gpu_rccl.py (not a test module): runs the SearchEngine round
protocol under a one-rank RCCL ("nccl") process group -- the all_gather of the scores
(search.py run_round) and the winner-image broadcast (_publish_best_image) really execute on the
GPU -- then the same searches with no process group, and prints one JSON line comparing them.
Started in a fresh process so that the process group is initialised before anything touches
the GPU (as bench.py / torchrun ranks do)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch
import torch.distributed as dist


def searches():
    from itsd.arch import ARCH_A
    from itsd.diffusion import GaussianDiffusionSampler
    from itsd.model import UNet
    from itsd.search import SearchEngine
    from itsd.verifier import OracleVerifier

    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss",
               device="cuda:0")
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, 20)
    eng = SearchEngine(smp, OracleVerifier(), seed=21)
    shape = (1, 3, 32, 32)
    out = {"dist": eng.dist, "world": eng.world}
    bn, bs, info = eng.random_search(8, shape)
    out["random"] = {"scores": info["scores"], "best_index": info["best_index"], "best_score": bs,
                     "best_noise": bn.cpu().flatten().tolist()[:64],
                     "best_image": eng.best_image.cpu().flatten().tolist()[:64]}
    init = eng.initial_noise(shape)
    bn, bs, h = eng.zero_order_search(init, 4, 0.95, 2)
    out["zo"] = {"scores": h["scores"], "best_score": bs, "best_noise": bn.cpu().flatten().tolist()[:64],
                 "best_image": eng.best_image.cpu().flatten().tolist()[:64]}
    del eng, smp, net
    torch.cuda.empty_cache()
    return out


def main():
    port = sys.argv[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    backend = dist.get_backend()
    with_group = searches()
    # one explicit collective of each kind the bench and the entry use, on device tensors
    t = torch.tensor([3.0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    dist.destroy_process_group()
    without = searches()
    same = {k: with_group[k] == without[k] for k in ("random", "zo")}
    print(json.dumps({"backend": backend, "dist_with": with_group["dist"], "dist_without": without["dist"],
                      "identical": same, "all_reduce": float(t.item()),
                      "random_best": with_group["random"]["best_index"]}), flush=True)


if __name__ == "__main__":
    main()
