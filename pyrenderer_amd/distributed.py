"""One process per GPU: interleaved tile sharding + RCCL gather.

Every rank renders the 64x64 tiles that device_scene.tile_owner assigns it (the
'latin' interleaving: tiles spread over every row and column of the frame, so
light-heavy and escape-heavy regions are shared evenly) into a device buffer of
per-tile radiance sums; the buffers are gathered to rank 0 with
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" on CPU
for tests) and rank 0 scatters the tiles into the (W, H, 3) frame.  Random
numbers are keyed by (seed, global pixel, sample), so the frame is
bit-identical for any world size.
"""
import numpy as np
import torch
import torch.distributed as dist

from .device_scene import interleaved_tiles, max_tiles_per_rank, tile_grid, unpack_tiles


class TileShard:
    """This rank's tiles and the padded gather buffers (allocated once).

    `buf` holds the rank's per-tile radiance sums on `device`.  With `host_staging` (the
    gloo backend, which moves CPU tensors) gather() first copies them to host memory."""

    def __init__(self, W, H, tile, rank, world, device, scheme="latin", host_staging=False):
        self.W, self.H, self.tile, self.rank, self.world = W, H, tile, rank, world
        self.scheme = scheme
        tx, ty = tile_grid(W, H, tile)
        self.n_tiles = tx * ty
        self.tiles = interleaved_tiles(W, H, tile, rank, world, scheme)
        self.max_tiles = max_tiles_per_rank(W, H, tile, world, scheme)
        self.slot_elems = tile * tile * 3
        self.buf = torch.zeros(self.max_tiles * self.slot_elems, dtype=torch.float32, device=device)
        self.host_staging = bool(host_staging) and self.buf.is_cuda
        self.wire = torch.empty_like(self.buf, device="cpu") if self.host_staging else self.buf
        self.gather_list = ([torch.empty_like(self.wire) for _ in range(world)]
                            if (world > 1 and rank == 0) else None)

    def gather(self, group=None):
        """Collective: rank 0 receives every rank's tile sums (no-op for world 1).  Runs on
        torch's current stream: callers that rendered on another stream enter it first."""
        if self.world > 1:
            if self.host_staging:
                self.wire.copy_(self.buf)       # synchronous device-to-host copy on the current stream
            dist.gather(self.wire, self.gather_list, dst=0, group=group)

    def assemble(self, device_scene=None, stream=None):
        """Rank 0: (W, H, 3) float32 sums frame from the gathered buffers.

        With `device_scene` (GPU ranks) the tiles are scattered into a device frame by libprt's
        scatter kernel (prt_scatter_tiles) on `stream` (default: torch's current stream) — the
        gathered buffers, already on the device over RCCL or uploaded once from gloo's host
        staging, never pass through a host loop; the frame is then copied to the host.  Without
        it (CPU-tensor shards: the gloo tests with the CPU oracle as renderer) the tiles are
        unpacked in numpy."""
        bufs = self.gather_list if self.world > 1 else [self.buf]
        per_rank = [interleaved_tiles(self.W, self.H, self.tile, r, self.world, self.scheme) for r in range(self.world)]
        if device_scene is None:
            frame = np.zeros((self.W, self.H, 3), np.float32)
            for b, ids in zip(bufs, per_rank):
                n = len(ids) * self.slot_elems
                unpack_tiles(b[:n].cpu().numpy().reshape(-1, 3), self.W, self.H, self.tile, self.tile, ids, frame)
            return frame
        dev = torch.device("cuda", device_scene.device)
        s = stream or torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            packed = torch.cat([b[:len(ids) * self.slot_elems].to(dev, non_blocking=False)
                                for b, ids in zip(bufs, per_rank)])
            frame = torch.zeros((self.W, self.H, 3), dtype=torch.float32, device=dev)
        ids = np.concatenate(per_rank).astype(np.int32)
        device_scene.scatter_tiles(packed.data_ptr(), ids, self.tile, self.tile, self.W, self.H, frame.data_ptr(),
                                   s.cuda_stream)
        with torch.cuda.stream(s):
            out = frame.cpu().numpy()
        return out


def render_distributed(device_scene, cam_packed, W, H, spp, depth, seed=0, tile=64, group=None, stream=None):
    """Render a frame across the ranks of `group` (default: the default group); returns mean
    radiance (W, H, 3) on rank 0 and None elsewhere.

    The render and the gather are ordered on `stream` (default: torch's current stream of the
    scene's device).  Before the gather every rank synchronises and reads its traversal
    watchdog (prt_check_faults); the flags are combined with a MAX all-reduce, so a fault on
    any rank raises PrtError on every rank instead of returning a silently invalid frame."""
    from ._native import PRT_ERR_INTERNAL, PrtError
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    dev = torch.device("cuda", device_scene.device)
    host = world > 1 and dist.get_backend(group) == "gloo"
    shard = TileShard(W, H, tile, rank, world, dev, host_staging=host)
    s = stream or torch.cuda.current_stream(dev)
    device_scene.render_tiles_device(cam_packed, W, H, tile, tile, shard.tiles, spp, depth, shard.buf.data_ptr(),
                                     s.cuda_stream, seed=seed)
    try:
        device_scene.check_faults()
        fault = 0
    except PrtError as e:
        if e.code != PRT_ERR_INTERNAL:
            raise
        fault = 1
    if world > 1:
        f = torch.tensor([fault], dtype=torch.int32, device="cpu" if host else dev)
        with torch.cuda.stream(s):
            dist.all_reduce(f, op=dist.ReduceOp.MAX, group=group)
        fault = int(f.item())
    if fault:
        raise PrtError(PRT_ERR_INTERNAL, "traversal watchdog tripped on "
                       + ("this rank" if world == 1 else "at least one rank") + "; the frame is invalid")
    with torch.cuda.stream(s):
        shard.gather(group)
    if rank != 0:
        return None
    return shard.assemble(device_scene, s) / np.float32(max(spp, 1))
