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

    `bufs[f]` holds the rank's per-tile radiance sums of frame f (of `frames`, the frames one
    render call produces: DeviceScene.render_frames_device) on `device`; `buf` is frame 0.  With
    `host_staging` (the gloo backend, which moves CPU tensors) gather() first copies them to host
    memory.

    `collective`: take the gather / root-scatter path even at world 1 (bench.py --force-collective:
    a one-rank process group runs the N > 1 step's RCCL code on one GPU); world > 1 always does."""

    def __init__(self, W, H, tile, rank, world, device, scheme="latin", host_staging=False, frames=1,
                 collective=False):
        self.W, self.H, self.tile, self.rank, self.world = W, H, tile, rank, world
        self.coll = world > 1 or bool(collective)
        self.scheme = scheme
        self.frames = int(frames)
        tx, ty = tile_grid(W, H, tile)
        self.n_tiles = tx * ty
        self.tiles = interleaved_tiles(W, H, tile, rank, world, scheme)
        self.max_tiles = max_tiles_per_rank(W, H, tile, world, scheme)
        self.slot_elems = tile * tile * 3
        self.bufs = torch.zeros((self.frames, self.max_tiles * self.slot_elems), dtype=torch.float32, device=device)
        self.buf = self.bufs[0]
        # floats between consecutive frames of `bufs` (the largest shard's slot, >= this rank's tiles):
        # the out_pitch of DeviceScene.render_frames_device into bufs
        self.pitch = int(self.bufs.shape[1])
        self.host_staging = bool(host_staging) and self.buf.is_cuda
        self.wire = torch.empty_like(self.bufs, device="cpu") if self.host_staging else self.bufs
        self.gathered = None
        if self.coll and rank == 0:
            # one contiguous receive buffer [rank][frame][slots]: a group's frames arrive in ONE
            # gather, and frame f's tiles of every rank sit at the same offsets from
            # gathered[0, f], rank r's block a stride of frames * max_tiles tiles further on
            self.gathered = torch.empty((world, self.frames, self.bufs.shape[1]), dtype=torch.float32,
                                        device=self.wire.device)
        self.per_rank = [interleaved_tiles(W, H, tile, r, world, scheme) for r in range(world)]
        # rank-major tile ids of the gather buffer, max_tiles per rank (padding id -1, dropped): the
        # scatter reads rank r's block at r * frames * pitch floats (prt_scatter_frames)
        ids = np.full((world, self.max_tiles), -1, np.int32)
        for r, t in enumerate(self.per_rank):
            ids[r, :len(t)] = t
        self.scatter_ids = ids.reshape(-1)
        self.frame_out = None    # rank 0's device frames (frames, W, H, 3), allocated by scatter()
        self.packed_dev = None   # gloo: the gathered host buffer's device copy

    def gather_list(self, n_frames=1):
        """Rank 0's receive views for a gather of frames 0 .. n_frames-1 (None elsewhere)."""
        return list(self.gathered[:, :n_frames].unbind(0)) if self.gathered is not None else None

    def gather(self, group=None, n_frames=1):
        """Collective: rank 0 receives every rank's tile sums of frames 0 .. n_frames-1 in ONE
        gather.  Runs on torch's current stream: callers that rendered on
        another stream enter it first (ProcessGroupNCCL's collective stream waits for the current
        one when the gather is enqueued, so the send follows the render).  The receive side is
        ordered explicitly: the gather is issued asynchronously and its work's wait() makes the
        current stream wait for the collective stream (nccl; gloo: the host waits), so a
        scatter_frames() enqueued next on this stream reads the received tiles.  No-op without the
        collective path (world 1)."""
        if self.coll:
            if self.host_staging:
                self.wire[:n_frames].copy_(self.bufs[:n_frames])   # synchronous device-to-host copy
            work = dist.gather(self.wire[:n_frames], self.gather_list(n_frames), dst=0, group=group, async_op=True)
            work.wait()

    @property
    def frame(self):
        return None if self.frame_out is None else self.frame_out[0]

    def scatter_frames(self, device_scene, stream=None, n_frames=1):
        """Rank 0 after gather(n_frames): every rank's tiles of frames 0 .. n_frames-1 -> the device
        frames frame_out[:n_frames], ONE launch (prt_scatter_frames over world x max_tiles slots per
        frame, ADVICE r04: not (world - 1) x frames of other frames' padding), enqueued on `stream`.
        This is the root-side step of SURVEY.md §8(e) that bench.py times inside every N > 1 step."""
        dev = torch.device("cuda", device_scene.device)
        s = stream or torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            if self.frame_out is None:
                self.frame_out = torch.zeros((self.frames, self.W, self.H, 3), dtype=torch.float32, device=dev)
            if not self.coll:
                packed, ids, group_pitch = self.bufs, self.per_rank[0], 0
            else:
                packed = self.gathered
                if not packed.is_cuda:
                    if self.packed_dev is None:
                        self.packed_dev = torch.empty_like(self.gathered, device=dev)
                    self.packed_dev.copy_(self.gathered)
                    packed = self.packed_dev
                ids, group_pitch = self.scatter_ids, self.frames * self.pitch
        group_tiles = self.max_tiles if self.coll else max(len(ids), 1)
        if len(ids):
            device_scene.scatter_frames(packed.data_ptr(), ids, group_tiles, group_pitch, self.tile, self.tile, self.W,
                                        self.H, n_frames, self.pitch, self.frame_out.data_ptr(), s.cuda_stream)
        return self.frame_out[:n_frames]

    def scatter(self, device_scene, stream=None, f=0):
        """Rank 0 after gather(): every rank's tiles of frame f -> the (W, H, 3) device frame
        `frame_out[f]` (one prt_scatter_frames launch from frame f's base), enqueued on `stream`
        (default: torch's current stream).  gloo's host buffer is first uploaded on that stream (once
        per group, with frame 0)."""
        dev = torch.device("cuda", device_scene.device)
        s = stream or torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            # the frames are zeroed once: every pixel belongs to exactly one tile, which every
            # scatter overwrites
            if self.frame_out is None:
                self.frame_out = torch.zeros((self.frames, self.W, self.H, 3), dtype=torch.float32, device=dev)
            if not self.coll:
                base, ids, group_pitch = self.bufs[f], self.per_rank[0], 0
            else:
                packed = self.gathered
                if not packed.is_cuda:
                    if self.packed_dev is None:
                        self.packed_dev = torch.empty_like(self.gathered, device=dev)
                    if f == 0:
                        self.packed_dev.copy_(self.gathered)
                    packed = self.packed_dev
                base, ids, group_pitch = packed[0, f], self.scatter_ids, self.frames * self.pitch
        group_tiles = self.max_tiles if self.coll else max(len(ids), 1)
        if len(ids):
            device_scene.scatter_frames(base.data_ptr(), ids, group_tiles, group_pitch, self.tile, self.tile, self.W,
                                        self.H, 1, self.pitch, self.frame_out[f].data_ptr(), s.cuda_stream)
        return self.frame_out[f]

    def assemble(self, device_scene=None, stream=None, f=0):
        """Rank 0: (W, H, 3) float32 sums of frame f (host) from the gathered buffers.

        With `device_scene` (GPU ranks): scatter() on `stream`, then one device-to-host copy of
        the frame — the gathered tiles never pass through a host loop.  Without it (CPU-tensor
        shards: the gloo tests with the CPU oracle as renderer) the tiles are unpacked in numpy."""
        if device_scene is None:
            bufs = [self.gathered[r, f] for r in range(self.world)] if self.coll else [self.bufs[f]]
            frame = np.zeros((self.W, self.H, 3), np.float32)
            for b, ids in zip(bufs, self.per_rank):
                n = len(ids) * self.slot_elems
                unpack_tiles(b[:n].cpu().numpy().reshape(-1, 3), self.W, self.H, self.tile, self.tile, ids, frame)
            return frame
        dev = torch.device("cuda", device_scene.device)
        s = stream or torch.cuda.current_stream(dev)
        if self.coll and not self.gathered.is_cuda and f != 0:
            self.scatter(device_scene, s, 0)    # uploads the gloo host buffer for this group
        frame = self.scatter(device_scene, s, f)
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
