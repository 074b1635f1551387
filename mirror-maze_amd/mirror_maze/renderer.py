"""Renderer: the reference's compute dispatch as a Python object over the C ABI.

Method names follow the reference's operator interface:
  * ``upload_scene``   — make_buf for buffers 1, 2, 3, 5, 6 (src/main.rs:725-730)
  * ``compute_shader`` — copy_to_buf(chunks) + dispatch_thread_groups
                         (src/main.rs:778-885, kernel src/shaders.metal:245-368)
  * ``read_texture``   — the screen texture the dispatch writes
  * ``trace_tile``     — the offline renderer's throughput entry point

Device buffers for ``trace_tile`` are torch tensors on the GPU (torch is the
device-memory/stream plumbing); the library enqueues on torch's current
stream so ordering with torch ops (e.g. an RCCL gather) is preserved.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib
from .scene import Scene


class Renderer:
    def __init__(self, device: int = 0):
        self._ctx = C.c_void_p()
        check(lib().mm_create(device, C.byref(self._ctx)))
        self.device = device
        self._view = None
        self._pinned_stream = False

    # -- lifecycle --------------------------------------------------------
    def close(self) -> None:
        if self._ctx:
            lib().mm_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        check(rc, self._ctx)

    def set_stream(self, stream=None) -> None:
        """Pin a torch.cuda.Stream (or raw hipStream_t int).  None = follow
        torch's current stream at every trace_tile call (the default)."""
        self._pinned_stream = stream is not None
        handle = _lib.MM_OWN_STREAM if stream is None else int(getattr(stream, "cuda_stream", stream))
        self._check(lib().mm_set_stream(self._ctx, handle))

    def own_stream(self):
        """Pin the context's own (library-created, non-blocking) stream and
        return it as a torch.cuda.ExternalStream, so torch ops can be ordered
        with this context's work.  Two contexts on their own streams run
        independent frames concurrently (the next frame's blocks fill the
        CUs the previous frame's tail leaves idle)."""
        import torch

        self.set_stream(_lib.MM_OWN_STREAM)
        h = C.c_void_p()
        self._check(lib().mm_get_stream(self._ctx, C.byref(h)))
        return torch.cuda.ExternalStream(h.value, device=torch.device(f"cuda:{self.device}"))

    def set_wave_timeline(self, buf=None) -> None:
        """Diagnostics: per-wave (entry, staged, exit, chunks) u64 records of
        the wave-persistent kernel into an int64 CUDA tensor of shape
        (n_waves, 4); None turns recording off."""
        if buf is None:
            self._check(lib().mm_set_wave_timeline(self._ctx, None, 0))
        else:
            self._check(lib().mm_set_wave_timeline(self._ctx, buf.data_ptr(), buf.shape[0]))

    def set_pipeline(self, pipe: int) -> None:
        self._check(lib().mm_set_pipeline(self._ctx, pipe))

    def set_option(self, key: int, value: int) -> None:
        self._check(lib().mm_set_option(self._ctx, key, value))

    def scene_info(self, key: int) -> float:
        """mm_scene_info: facts about the uploaded scene's search structures
        (MM_INFO_*: grid availability and size, BVH depth)."""
        v = C.c_double()
        self._check(lib().mm_scene_info(self._ctx, key, C.byref(v)))
        return v.value

    # -- scene ------------------------------------------------------------
    def upload_scene(self, s: Scene) -> None:
        rects = np.ascontiguousarray(s.rects, dtype=np.float32)
        nodes = np.ascontiguousarray(s.nodes)
        idx = np.ascontiguousarray(s.idx, dtype=np.uint32)
        mats = np.ascontiguousarray(s.is_mirror, dtype=np.uint8)
        emis = np.ascontiguousarray(s.emission, dtype=np.float32)
        self._check(lib().mm_upload_scene(self._ctx, rects.ctypes.data, rects.shape[0], nodes.ctypes.data,
                                          nodes.shape[0], idx.ctypes.data, mats.ctypes.data, emis.ctypes.data))

    # -- parity mode --------------------------------------------------------
    def compute_shader(self, uniform: _lib.mm_uniform, pixel_update_buffer: np.ndarray) -> None:
        """One reference dispatch: (W/32)x(H/32) groups, 64 samples per pixel."""
        chunks = np.ascontiguousarray(pixel_update_buffer, dtype=np.uint32).reshape(-1, 2)
        self._check(lib().mm_trace_chunks(self._ctx, C.byref(uniform), chunks.ctypes.data, chunks.shape[0]))
        self._view = (int(uniform.view_w), int(uniform.view_h))

    def read_texture(self):
        """(rgba_f32 [H,W,4], rgba8 [H,W,4]) of the screen texture."""
        if self._view is None:
            raise RuntimeError("nothing rendered yet")
        W, H = self._view
        f = np.zeros((H, W, 4), dtype=np.float32)
        b = np.zeros((H, W, 4), dtype=np.uint8)
        self._check(lib().mm_read_framebuffer(self._ctx, f.ctypes.data, b.ctypes.data))
        return f, b

    def present(self) -> None:
        """One presentation step: the fragment_shader blur of the RGBA8 texture
        as a Jacobi step (src/shaders.metal:214-225; mm_present)."""
        self._check(lib().mm_present(self._ctx))

    def read_packets(self, n_chunks: int) -> np.ndarray:
        """(n_chunks, 16, 4) float32 packets of the last compute_shader: rgb and
        bitcast(x << 16 | y) (the shaders.air revision's pixel_data output)."""
        out = np.zeros((n_chunks, 16, 4), dtype=np.float32)
        self._check(lib().mm_read_packets(self._ctx, out.ctypes.data, n_chunks))
        return out

    def quantize(self, rgba, out=None):
        """RGBA8 (uint8 CUDA tensor, same shape; into `out` if given) of a float32
        RGBA CUDA tensor, with the texture-write conversion (mm_quantize_rgba8)."""
        import torch

        if not (rgba.is_cuda and rgba.dtype == torch.float32 and rgba.is_contiguous() and rgba.shape[-1] == 4):
            raise ValueError("rgba must be a contiguous float32 CUDA tensor [..., 4]")
        if out is None:
            out = torch.empty(rgba.shape, dtype=torch.uint8, device=rgba.device)
        elif not (out.is_cuda and out.dtype == torch.uint8 and out.is_contiguous() and out.shape == rgba.shape):
            raise ValueError("out must be a contiguous uint8 CUDA tensor of rgba's shape")
        if not self._pinned_stream:
            self._check(lib().mm_set_stream(self._ctx, torch.cuda.current_stream(rgba.device).cuda_stream))
        self._check(lib().mm_quantize_rgba8(self._ctx, rgba.data_ptr(), out.data_ptr(), rgba.numel() // 4))
        return out

    # -- throughput mode ------------------------------------------------------
    @staticmethod
    def _out(out, shape, rgba8, device):
        """The output tensor: float32 (..., 4), or uint8 (..., 4) for RGBA8
        frames (MM_EXT_RGBA8, set when `out` is uint8 or rgba8=True)."""
        import torch

        if out is None:
            out = torch.zeros(shape, dtype=torch.uint8 if rgba8 else torch.float32, device=device)
        n = 1
        for d in shape:
            n *= d
        if not (out.is_cuda and out.dtype in (torch.float32, torch.uint8) and out.is_contiguous()
                and out.numel() == n):
            raise ValueError(f"out must be a contiguous float32 or uint8 CUDA tensor of {n} elements")
        return out, out.dtype == torch.uint8

    def trace_tile(self, uniform: _lib.mm_uniform, ext: _lib.mm_ext, x0: int, y0: int, w: int, h: int,
                   y_stride: int = 1, out=None, stats: bool = False, rgba8: bool = False):
        """Render a tile into a (h, w, 4) float32 CUDA tensor (allocated if None),
        or with rgba8 / a uint8 `out` its RGBA8 texture-write conversion
        (MM_EXT_RGBA8: equal to quantize() of the float tile).  Returns (out,
        mm_stats or None)."""
        import torch

        out, r8 = self._out(out, (h, w, 4), rgba8, f"cuda:{self.device}")
        if not self._pinned_stream:  # order with the torch ops that made / read `out`
            self._check(lib().mm_set_stream(self._ctx, torch.cuda.current_stream(out.device).cuda_stream))
        e = _lib.mm_ext(ext.spp, ext.bounce_limit, ext.mirror_limit, ext.frame,
                        ext.flags | (_lib.MM_EXT_COUNT_STATS if stats else 0) | (_lib.MM_EXT_RGBA8 if r8 else 0), 0)
        st = _lib.mm_stats()
        self._check(lib().mm_trace_tile(self._ctx, C.byref(uniform), C.byref(e), x0, y0, w, h, y_stride,
                                        out.data_ptr(), C.byref(st)))
        return out, (st if stats else None)

    def trace_tile_frames(self, uniform: _lib.mm_uniform, ext: _lib.mm_ext, n_frames: int, x0: int, y0: int,
                          w: int, h: int, y_stride: int = 1, out=None, stats: bool = False, rgba8: bool = False):
        """Render frames ext.frame .. ext.frame + n_frames - 1 of a tile in ONE
        launch (mm_trace_tile_frames) into a (n_frames, h, w, 4) float32 CUDA
        tensor (allocated if None; uint8 RGBA8 with rgba8 / a uint8 `out`, as
        trace_tile); frame f equals trace_tile with frame ext.frame + f.
        Returns (out, mm_stats summed over the frames or None)."""
        import torch

        out, r8 = self._out(out, (n_frames, h, w, 4), rgba8, f"cuda:{self.device}")
        if not self._pinned_stream:
            self._check(lib().mm_set_stream(self._ctx, torch.cuda.current_stream(out.device).cuda_stream))
        e = _lib.mm_ext(ext.spp, ext.bounce_limit, ext.mirror_limit, ext.frame,
                        ext.flags | (_lib.MM_EXT_COUNT_STATS if stats else 0) | (_lib.MM_EXT_RGBA8 if r8 else 0), 0)
        st = _lib.mm_stats()
        self._check(lib().mm_trace_tile_frames(self._ctx, C.byref(uniform), C.byref(e), n_frames, x0, y0, w, h,
                                               y_stride, out.data_ptr(), C.byref(st)))
        return out, (st if stats else None)

    def sync(self) -> None:
        """Wait for this context's work; raises MMError for the oldest
        trace_tile* call that failed on the GPU and was not reported yet (the
        message names that call)."""
        self._check(lib().mm_sync(self._ctx))

    def last_call(self) -> int:
        """Number of the last trace_tile / trace_tile_frames call (1, 2, ...)."""
        n = C.c_uint64()
        self._check(lib().mm_last_call(self._ctx, C.byref(n)))
        return n.value

    def call_status(self, call_id: int) -> bool:
        """Without waiting: True if call `call_id` finished clean, False while
        it runs; raises MMError (naming the call) if it failed on the GPU."""
        rc = lib().mm_call_status(self._ctx, call_id)
        if rc == _lib.MM_PENDING:
            return False
        self._check(rc)
        return True

    def set_profiling(self, enable: bool = True) -> None:
        self._check(lib().mm_set_profiling(self._ctx, 1 if enable else 0))

    def kernel_timing(self, reset: bool = True):
        """(summed ms, launches) of the ray-trace kernel since the last reset."""
        ms, n = C.c_float(), C.c_uint32()
        self._check(lib().mm_kernel_timing(self._ctx, C.byref(ms), C.byref(n), 1 if reset else 0))
        return ms.value, n.value

    def last_timing(self):
        ms, n = C.c_float(), C.c_uint32()
        self._check(lib().mm_last_timing(self._ctx, C.byref(ms), C.byref(n)))
        return ms.value, n.value


def make_ext(spp: int = 8, bounce_limit: int = 8, mirror_limit: int = 8, frame: int = 0,
             flags: int = 0) -> _lib.mm_ext:
    return _lib.mm_ext(spp, bounce_limit, mirror_limit, frame, flags, 0)
