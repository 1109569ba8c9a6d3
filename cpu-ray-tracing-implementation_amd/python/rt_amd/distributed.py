"""One frame over the ranks of a process group (replaces the reference's per-row
std::execution::par loop, camera.h:154-172): every rank renders its 16x16 tiles (tiling.plan,
dealt round-robin) into a padded device buffer through the C ABI, rank 0 gathers the buffers and
scatters them into the linear framebuffer.

The gather is the only exchange. With the "nccl" backend (RCCL over xGMI on ROCm) it moves the
device buffers; with "gloo" (CPU rehearsals, or several ranks sharing one GPU in the -m gpu test)
the buffers go through host memory. The image does not depend on the rank count: every sample's
random numbers are keyed by (seed, global pixel, sample) and the item layout by spp alone.
"""
import torch
import torch.distributed as dist

from .abi import TileList
from .tiling import pixel_index, plan


class FrameSharding:
    """The tile plan of one rank and, on rank 0, the scatter indices of every rank's packed pixels."""

    def __init__(self, width, height, world, rank, device, group=None):
        self.W, self.H, self.world, self.rank, self.device, self.group = width, height, world, rank, device, group
        self.tiles, self.counts, self.maxpix = plan(width, height, world)
        self.my_tiles = self.tiles[rank]
        self._my_tiles_c = TileList(self.my_tiles)  # the ctypes form, built once (render_tiles)
        self.backend = dist.get_backend(group) if world > 1 else None
        self.scatter_idx = None
        self._recv = {}  # rank 0's gather buffers, per (dtype, device), reused frame to frame
        if rank == 0:
            self.scatter_idx = [torch.from_numpy(pixel_index(self.tiles[r], width)).to(device) for r in range(world)]

    def buffers(self, dtype):
        """(this rank's padded tile buffer, rank 0's framebuffer or None), on the device."""
        out = torch.zeros((self.maxpix, 3), dtype=dtype, device=self.device)
        fb = torch.zeros((self.H * self.W, 3), dtype=dtype, device=self.device) if self.rank == 0 else None
        return out, fb

    def frame(self, ctx, cam, params, out, fb, stream=None):
        """Render this rank's tiles into `out`, gather every rank's buffer to rank 0 and scatter them into
        `fb` (rank 0). The render is queued on `stream` (a torch.cuda.Stream; default torch's current
        stream). The gather and the scatter are ordered against torch's current stream, so a render on
        another stream is joined to it by an event first."""
        if stream is None:
            handle = torch.cuda.current_stream(self.device).cuda_stream
            ctx.render_tiles(cam, params, self._my_tiles_c, out.data_ptr(), 1, handle)
        elif isinstance(stream, torch.cuda.Stream):
            ctx.render_tiles(cam, params, self._my_tiles_c, out.data_ptr(), 1, stream.cuda_stream)
            cur = torch.cuda.current_stream(self.device)
            if stream != cur:
                ev = torch.cuda.Event()
                ev.record(stream)
                cur.wait_event(ev)
        else:  # a raw handle: only the current stream's (or 0 for a CPU rehearsal without a GPU) is ordered
            if torch.cuda.is_available() and stream not in (0, torch.cuda.current_stream(self.device).cuda_stream):
                raise ValueError("pass a torch.cuda.Stream: a raw handle of another stream cannot be ordered "
                                 "before the gather")
            ctx.render_tiles(cam, params, self._my_tiles_c, out.data_ptr(), 1, stream)
        if self.world == 1:
            parts = [out]
        elif self.backend == "gloo":  # host-memory gather (the device buffer is copied behind the render)
            host = out.cpu()
            parts = self._parts(host)
            dist.gather(host, parts, dst=0, group=self.group)
        else:  # RCCL: the device buffers, stream-ordered behind the render
            parts = self._parts(out)
            dist.gather(out, parts, dst=0, group=self.group)
        if self.rank == 0:
            for r in range(self.world):
                fb[self.scatter_idx[r]] = parts[r][: self.counts[r]].to(self.device, non_blocking=True)

    def _parts(self, like):
        if self.rank != 0:
            return None
        key = (like.dtype, like.device)
        if key not in self._recv:
            self._recv[key] = [torch.empty_like(like) for _ in range(self.world)]
        return self._recv[key]
