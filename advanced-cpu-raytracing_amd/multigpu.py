"""Image partition across the GPUs of one node, and the host framebuffer gather.

The reference's only parallelism is row bands over std::threads (src/main.cpp:38-39,
164-185: thread t renders rows [t*H/8, (t+1)*H/8)).  Here the frame is dealt to GPUs in
8-row bands (RTG_PART_BAND_ROWS, the rows of one wave's 8x8 pixel block), dealt round-robin
with the order rotated by one slot per round: the k-th band of part p is band
k * N + ((p - k) mod N).  Interleaving the bands balances the image's cost gradient over the
parts, and the rotation its gradient within a round of N bands (a
contiguous band per GPU would not -- the CPU shows 1->8 threads giving only 2.5x on
ton_Roosendaal), and every band is a contiguous run of the row-major
framebuffer (layout 3*(x + y*W), main.cpp:109), so the gather is one DMA per run straight
into the final frame: no collective, no host-side re-tiling.

Two ways to drive it, both bit-identical to a single-GPU render (pixels are independent
and the RNG is keyed by pixel / sample / ray-tree node, never by device):

* one process, several GPUs: ``rtgpu.DeviceScene(host, devices=[0, 1, ...])``
  (rtg_scene_create_multi) -- ``render()`` deals the parts to the replicas' streams and
  copies each part into the caller's frame (what the CLI's ``--devices`` uses);
* one process per GPU (torch.distributed launch, bench.py): rank r renders part r of N
  with ``DeviceScene.render_device(..., part=(r, N))`` into its own HBM, and
  ``copy_part_to_host`` DMAs its rows into a ``SharedFrame`` -- one page-locked
  shared-memory framebuffer mapped by every rank on the node; after a barrier
  ``finish_frame`` tonemaps the gathered frame on rank 0 for a <Tonemap> camera.

``sample_range`` (sample-parallel split with host accumulation) is kept for
multi-sample cameras whose frame is too small to cut.
"""
from __future__ import annotations

import ctypes
import mmap
import os

import numpy as np

BAND_ROWS = 8    # RTG_PART_BAND_ROWS (include/rtgpu.h)


def part_runs(row_begin: int, row_end: int, part: int, parts: int):
    """Rows of part ``part`` of ``parts`` in [row_begin, row_end) as maximal runs
    [(r0, r1), ...] -- the library's own arithmetic (rtg_part_runs, host-only)."""
    import rtgpu
    L = rtgpu.lib()
    n = ctypes.c_int32()
    rtgpu._check(L.rtg_part_runs(row_begin, row_end, part, parts, None, 0, ctypes.byref(n)))
    buf = (ctypes.c_int32 * (2 * max(1, n.value)))()
    rtgpu._check(L.rtg_part_runs(row_begin, row_end, part, parts, buf, n.value, ctypes.byref(n)))
    return [(buf[2 * k], buf[2 * k + 1]) for k in range(n.value)]


def part_runs_py(row_begin: int, row_end: int, part: int, parts: int):
    """Pure-Python statement of the same partition (cross-check of rtg_part_runs)."""
    runs = []
    parts = max(parts, 1)
    k = 0
    while True:
        b = k * parts + (part - k) % parts       # round-robin, rotated one slot per round
        a = row_begin + b * BAND_ROWS
        if a >= row_end:
            return runs
        e = min(a + BAND_ROWS, row_end)
        if runs and runs[-1][1] == a:
            runs[-1] = (runs[-1][0], e)
        else:
            runs.append((a, e))
        k += 1


def sample_range(rank: int, world: int, spp: int):
    """Contiguous samples [begin, begin+count) of rank ``rank`` among ``world``."""
    base, extra = divmod(spp, world)
    begin = rank * base + min(rank, extra)
    return begin, base + (1 if rank < extra else 0)


class SharedFrame:
    """One host framebuffer shared by the ranks of a node: a /dev/shm file mapped by every
    process (rank 0 creates it, the others attach after a barrier), holding the float image
    (W*H*3 f32, main.cpp:114-116) and/or the 8-bit image (W*H*3 u8, main.cpp:121) in the
    reference's layout.  ``pin()`` page-locks the mapping for this process's HIP runtime
    (rtg_host_register) so each rank's part copy is an asynchronous DMA into its rows."""

    def __init__(self, name: str, height: int, width: int, hdr: bool = True, ldr: bool = True,
                 create: bool = False):
        self.path = os.path.join("/dev/shm", name)
        self.h, self.w = height, width
        n = height * width * 3
        self.hdr_bytes = 4 * n if hdr else 0
        self.ldr_bytes = n if ldr else 0
        size = max(1, self.hdr_bytes + self.ldr_bytes)
        size = (size + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
        flags = os.O_RDWR | (os.O_CREAT if create else 0)
        fd = os.open(self.path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, size)
            self._mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.size = size
        self.owner = create
        buf = np.frombuffer(self._mm, np.uint8)
        self.hdr = buf[:self.hdr_bytes].view(np.float32).reshape(height, width, 3) if hdr else None
        self.ldr = buf[self.hdr_bytes:self.hdr_bytes + self.ldr_bytes].reshape(height, width, 3) if ldr else None
        self._pinned = False

    def base_ptr(self) -> int:
        return ctypes.addressof(ctypes.c_char.from_buffer(self._mm))

    def hdr_ptr(self) -> int:
        return self.base_ptr() if self.hdr is not None else 0

    def ldr_ptr(self) -> int:
        return self.base_ptr() + self.hdr_bytes if self.ldr is not None else 0

    def pin(self):
        import rtgpu
        rtgpu._check(rtgpu.lib().rtg_host_register(self.base_ptr(), self.size))
        self._pinned = True

    def close(self):
        if self._pinned:
            import rtgpu
            rtgpu.lib().rtg_host_unregister(self.base_ptr())
            self._pinned = False
        self.hdr = self.ldr = None
        if self._mm is not None:
            try:
                self._mm.close()
            except BufferError:      # a numpy view still alive: the mapping goes with it
                pass
            self._mm = None
        if self.owner and os.path.exists(self.path):
            os.unlink(self.path)


def render_part(ds, rank: int, world: int, d_hdr: int, d_ldr: int, stream: int, frame: SharedFrame | None = None,
                camera: int = 0, seed: int = 0x5EED, flags: int = 0, overlap: bool = True):
    """Rank ``rank``'s share of one frame.

    With a ``frame`` and ``overlap`` (the default): rtg_render of part rank/world straight into
    the shared page-locked host framebuffer -- the kernels write the part's pixels over the bus
    as they render, so no copy follows.  Synchronous; ``stream``, ``d_hdr`` and
    ``d_ldr`` are unused.  (RTG_HOST_CHUNKS=1 opts into rendering the part in row chunks on two
    streams with each chunk's DMA overlapping the next chunk: measured slower, rtg_api.cpp
    render_chunked.)
    Otherwise: render the part into its device buffers (full-frame sized; only its rows are
    written) and, with a ``frame``, enqueue the DMA of those rows into the shared host
    framebuffer after it.  Asynchronous on ``stream``."""
    if frame is not None and overlap:
        ds.render(camera, flags=flags, seed=seed, part=(rank, world), out=(frame.hdr, frame.ldr))
        return
    ds.render_device(d_hdr, d_ldr, stream, camera=camera, seed=seed, flags=flags, part=(rank, world))
    if frame is not None:
        ds.copy_part_to_host(d_hdr if frame.hdr is not None else 0, d_ldr if frame.ldr is not None else 0,
                             frame.hdr_ptr(), frame.ldr_ptr(), stream, camera=camera, part=(rank, world))


def finish_frame(host, frame: SharedFrame, camera: int = 0, rank: int = 0, device: int = 0) -> bool:
    """After every rank's part has landed in ``frame`` (a barrier): a camera with a <Tonemap>
    needs the whole frame (the log-average and the burn percentile are over all pixels,
    tonemapper.h:28-60), so rank 0 tonemaps the gathered float image into the frame's LDR,
    as main.cpp:187-192 does after its threads join.  The parts' own LDR rows hold the
    un-tonemapped clamp until then.  Returns True when it tonemapped."""
    params = host.tonemap_params(camera)
    if params is None or rank != 0:
        return False
    if frame.hdr is None or frame.ldr is None:
        raise ValueError("a tonemapped camera's shared frame needs both the float and the 8-bit image")
    import rtgpu
    frame.ldr[...] = rtgpu.tonemap(frame.hdr, *params, device=device)
    return True

