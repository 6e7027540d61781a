"""Multi-GPU: image row stripes across one process per GPU.

Pixels are independent in the reference (per-pixel seed chain, history and
count; read-only scene), so rank r renders the 16-row stripes s with
s % world == r and no data moves during the frame loop.  At the end the
zero-elsewhere accumulators (mean, count, seed: 24 B per pixel) are packed
into one flat int32 buffer and summed onto rank 0 by ONE reduce (RCCL over
xGMI with the nccl backend; gloo on CPU in tests).  Each pixel has exactly
one non-zero contributor, so the integer sum of bit patterns is that
contributor's bits — exact for floats too, -0.0 included — giving the
single-GPU image for any GPU count.
"""
import numpy as np
import torch
import torch.distributed as dist


def owned_rows(height, stripe_rows, rank, world):
    """Rows of this rank, in the kernel's local-row order (k_render's global_row)."""
    rows = []
    lr = 0
    while True:
        s = lr // stripe_rows
        y = (s * world + rank) * stripe_rows + lr % stripe_rows
        if y >= height:
            break
        rows.append(y)
        lr += 1
    return np.asarray(rows, np.int64)


def owned_pixels(width, height, stripe_rows, rank, world):
    rows = owned_rows(height, stripe_rows, rank, world)
    return (rows[:, None] * width + np.arange(width)[None, :]).reshape(-1)


def ownership_mask(width, height, stripe_rows, rank, world):
    m = np.zeros(width * height, bool)
    m[owned_pixels(width, height, stripe_rows, rank, world)] = True
    return m


def reduce_image(hist, count, seeds, mask, group=None, dst=0):
    """Sum every rank's owned pixels onto rank `dst` with one collective.

    hist (N,4) float32, count (N,) int32, seeds (N,) int32 view of u32 — any
    device the process group's backend supports.  Non-owned pixels are zeroed,
    the three arrays packed as int32 bit patterns into one (N, 6) buffer and
    reduced with an integer SUM (one contributor per pixel: exact bits).
    Returns (hist float32 (N,4), count int32, seeds int64 holding the u32)."""
    if hist.is_cuda and dist.get_backend(group) == "gloo":  # gloo reduces host tensors
        hist, count, seeds = hist.cpu(), count.cpu(), seeds.cpu()
    m = torch.as_tensor(mask, device=hist.device)
    flat = torch.empty((hist.shape[0], 6), dtype=torch.int32, device=hist.device)
    flat[:, :4] = hist.contiguous().view(torch.int32)
    flat[:, 4] = count
    flat[:, 5] = seeds.view(torch.int32) if seeds.dtype == torch.int32 else seeds.to(torch.int32)
    flat.masked_fill_(~m[:, None], 0)
    dist.reduce(flat, dst=dst, op=dist.ReduceOp.SUM, group=group)
    h = flat[:, :4].contiguous().view(torch.float32)
    return h, flat[:, 4].contiguous(), flat[:, 5].to(torch.int64) & 0xFFFFFFFF


def render_distributed(renderer, scene, camera, width, height, max_depth, max_attempt, frames, seeds,
                       stripe_rows=16, group=None, mode=0):
    """Render the whole image across the process group; rank 0 gets the image.
    Returns (hist, count, seeds) as numpy on rank 0, None elsewhere."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    st = renderer.new_state(width, height, seeds)
    kw = dict(stripe_rows=stripe_rows, stripe_index=rank, stripe_count=world, mode=mode)
    if frames >= 4096:  # long runs: each rank times the leaf schedules and S/fetch thresholds on one-block
        # 16-frame calls (same bits; neither block sizing nor tile order is tuned: long calls run
        # max_block_frames blocks, a regime one-block trials do not enter, App.update)
        renderer.tune(scene, camera, st, max_depth, max_attempt, frames=16, block_entries=None, last_block=False,
                      tile_orders=None, frames_per_launch=16, **kw)
    renderer.render_frames(scene, camera, st, max_depth, max_attempt, frames, **kw)
    torch.cuda.synchronize()
    mask = ownership_mask(width, height, stripe_rows, rank, world)
    h, c, s = reduce_image(st.hist, st.count, st.seeds, mask, group=group)
    if rank != 0:
        return None
    return h.cpu().numpy(), c.cpu().numpy(), s.cpu().numpy().astype(np.uint32)
