"""Worker for the world_size>1 gloo tests (imported by spawned processes)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "capnproto-rust_amd"))


def batch(seed=11, n=400):
    import oracle_lib as O
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, 700, n)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    kinds = rng.integers(0, 3, n).astype(np.uint8)
    words = O.gen_fill(offs, kinds=kinds, pz=O.PZ30)
    return words, offs


def pack_concat_worker(rank, world, port, outdir):
    """Each rank packs its word-balanced shard (CPU oracle standing in for
    the device codec), the ranks exchange shard totals, and the concatenated
    stream and offsets are written for the parent to check."""
    import torch.distributed as dist
    import oracle_lib as O
    from capnp_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    words, offs = batch()
    b = shard.shard_by_words(offs, world)
    c0, c1 = b[rank], b[rank + 1]
    local_offs = (offs[c0:c1 + 1] - offs[c0]).astype(np.uint64)
    st, packed, loff = O.pack_batch(words[int(offs[c0]):int(offs[c1])], local_offs)
    assert st == 0
    totals = shard.gather_totals(int(loff[-1]))
    starts = shard.exclusive_offsets(totals)
    goff = shard.global_chunk_offsets(loff, starts[rank])
    elapsed = shard.max_over_ranks(0.5 + rank)
    np.save(os.path.join(outdir, f"packed{rank}.npy"), packed)
    np.save(os.path.join(outdir, f"offs{rank}.npy"), goff)
    with open(os.path.join(outdir, f"meta{rank}.txt"), "w") as f:
        f.write(f"{c0} {c1} {starts[rank]} {starts[-1]} {elapsed}\n")
    dist.barrier()
    dist.destroy_process_group()


def pack_concat_worker_gpu(rank, world, port, outdir):
    """The same assembly with the device codec: every rank packs its shard
    on cuda:0 through the C ABI (a one-GPU box runs the ranks side by side
    on its one device), the ranks exchange shard totals over gloo, and the
    concatenated stream and offsets are written for the parent to check."""
    import torch
    import torch.distributed as dist
    from capnp_amd import Context, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ctx = Context(0)
    words, offs = batch(seed=23, n=3000)
    b = shard.shard_by_words(offs, world)
    c0, c1 = b[rank], b[rank + 1]
    local_offs = (offs[c0:c1 + 1] - offs[c0]).astype(np.int64)
    dw = torch.from_numpy(words[int(offs[c0]):int(offs[c1])].view(np.int64).copy()).cuda()
    do = torch.from_numpy(local_offs).cuda()
    packed, loff = ctx.pack_batch(dw, do)
    torch.cuda.synchronize()
    packed = packed.cpu().numpy()
    loff = loff.cpu().numpy().view(np.uint64)
    totals = shard.gather_totals(int(loff[-1]))
    starts = shard.exclusive_offsets(totals)
    goff = shard.global_chunk_offsets(loff, starts[rank])
    np.save(os.path.join(outdir, f"packed{rank}.npy"), packed)
    np.save(os.path.join(outdir, f"offs{rank}.npy"), goff)
    with open(os.path.join(outdir, f"meta{rank}.txt"), "w") as f:
        f.write(f"{c0} {c1} {starts[rank]} {starts[-1]}\n")
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()
