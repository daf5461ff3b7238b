"""Host-side mirror of the reference's `RaytracingMaster` MonoBehaviour
(Assets/Scripts/SVO/GPU/RaytracingMaster.cs) over the C-ABI of libsvo_rt.so.

Same names and argument meaning as the reference:
  InitializeSVOBuffer()          RaytracingMaster.cs:111-116
  SetSVOBuffer(data, offset=0)   RaytracingMaster.cs:118-135 (public overload)
  SetSVOBuffer()                 RaytracingMaster.cs:90-109  (rebuild from maxLevel / sampleType)
  UpdateShaderParameters(...)    RaytracingMaster.cs:32-41
  Render(width, height)          RaytracingMaster.cs:60-74   (Dispatch + result)
  accumulate_device(...)         RaytracingMaster.cs:70-73 + AddShader.shader (Blit with _Sample,
                                 then _currentSample++; reset to 0 when the camera moves, :44-47)
  RenderProgressive(width, height)  OnRenderImage end to end (:55-74): one sample rendered,
                                 accumulated on the device, display RGBA8 to the host
Beyond the reference (one GPU, one Dispatch):
  RaytracingMaster(devices=[0, 1, ...])  one context over several GPUs of the node
                                 (svo_create_multi): SVO replica per GPU, the frame
                                 rendered in row bands and gathered to devices[0]
  render_frame(...)              every per-pixel output (hits, Result, RGBA8,
                                 compact records, hit position, voxel key)
  assemble_frame(...)            rebuild a frame from band parts (the display side
                                 of the one-process-per-GPU split)
Errors surface as SvoError (the C-ABI status + svo_last_error text) instead of
Unity's silent shader failures.  There is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import HIT_DTYPE, LAYOUT_BAND, LAYOUT_FRAME, STACK_EXACT, STACK_HLSL, SvoError, SvoFrame, check, make_band
from .camera import column_major, main_camera, main_light
from .svo_data import SVOData

# RaytracingMaster.cs:113-115: "one gibibyte of memory" / 8 elements of 4 bytes
REFERENCE_CAPACITY = 1073741824 // 8


def _frame(hits=None, rgba=None, rgba8=None, compact=None, position=None, voxel=None, layout=LAYOUT_BAND, rgb8=None,
           hitmask=None):
    return SvoFrame(hits, rgba, rgba8, compact, position, voxel, rgb8, hitmask, layout)


class RaytracingMaster:
    def __init__(self, device=0, capacity_nodes=REFERENCE_CAPACITY, maxLevel=5, sampleType=4, devices=None,
                 band_rows=8, config=None):
        """devices: list of HIP device indices for a multi-device context (devices[0]
        displays; an index may repeat); None = the single device `device`.
        config: svo_config fields to set on the new context (set_config)."""
        self.devices = None if devices is None else [int(d) for d in devices]
        self.device = device if devices is None else self.devices[0]
        self.band_rows = int(band_rows)
        self.capacity_nodes = int(capacity_nodes)
        self.maxLevel = maxLevel        # [Range(1, 8)] in the reference (:16-17)
        self.sampleType = sampleType    # SampleFunctions.Type.Custom1 = 4 (:18)
        self._ctx = ctypes.c_void_p()
        self._camera_set = False
        self._c2w = None
        self._options = 0               # svo_set_options bits
        self.currentSample = 0          # _currentSample (RaytracingMaster.cs:12)
        self._config = dict(config or {})
        self.InitializeSVOBuffer()

    # ------------------------------------------------------------------ setup
    def InitializeSVOBuffer(self):
        L = _lib.lib()
        if self._ctx:
            L.svo_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()
        if self.devices is None:
            check(L.svo_create(self.device, self.capacity_nodes, ctypes.byref(self._ctx)), "svo_create")
        else:
            arr = (ctypes.c_int * len(self.devices))(*self.devices)
            check(L.svo_create_multi(arr, len(self.devices), self.capacity_nodes, self.band_rows,
                                     ctypes.byref(self._ctx)), "svo_create_multi")
        self._options = 0
        if self._config:
            self.set_config(**self._config)

    def get_config(self):
        """The context's svo_config (render policy) as a dict."""
        c = _lib.SvoConfig()
        c.size = ctypes.sizeof(_lib.SvoConfig)
        check(_lib.lib().svo_get_config(self._ctx, ctypes.byref(c)), "svo_get_config")
        return c.to_dict()

    def set_config(self, **fields):
        """Change svo_config fields (include/svo_rt.h; the counterpart of RaytracingMaster's Inspector
        fields, RaytracingMaster.cs:16-18): the others keep their values.  Policy only -- every
        setting renders the same frames."""
        c = _lib.SvoConfig()
        c.size = ctypes.sizeof(_lib.SvoConfig)
        check(_lib.lib().svo_get_config(self._ctx, ctypes.byref(c)), "svo_get_config")
        names = {n for n, _ in _lib.CONFIG_FIELDS}
        for k, v in fields.items():
            if k not in names:
                raise SvoError(f"svo_config has no field {k!r}")
            setattr(c, k, v)
        check(_lib.lib().svo_set_config(self._ctx, ctypes.byref(c)), "svo_set_config")
        self._config.update(fields)

    def SetSVOBuffer(self, data=None, offset=0):
        """Upload an SVOData at descriptor `offset`; with no data, build one from
        (sampleType, maxLevel) like the private reference overload."""
        if data is None:
            from .builder import build_svo_for_sampler
            data = build_svo_for_sampler(self.sampleType, self.maxLevel)
        if not isinstance(data, SVOData):
            raise TypeError("SetSVOBuffer expects an SVOData")
        L = _lib.lib()
        att = np.ascontiguousarray(data.attachments, np.uint32)
        if data.format == 1:
            desc = np.ascontiguousarray(data.childDescriptors, np.int32)
            check(L.svo_set_buffer(self._ctx, desc.ctypes.data, len(desc), att.ctypes.data, len(att), int(offset)),
                  "svo_set_buffer")
        else:
            nodes = np.ascontiguousarray(data.nodes, np.uint64)
            check(L.svo_set_buffer_v2(self._ctx, nodes.ctypes.data, len(nodes), att.ctypes.data, len(att),
                                      int(offset)), "svo_set_buffer_v2")
        return data

    def UpdateShaderParameters(self, camera=None, width=1920, height=1080, pixel_offset=(0.5, 0.5), light=None):
        """camera: raytracingtest_amd.camera.Camera, or a (c2w, inv_proj) pair of 4x4 arrays."""
        camera = main_camera() if camera is None else camera
        if isinstance(camera, tuple):
            c2w, inv_proj = camera
        else:
            c2w, inv_proj = camera.uniforms(width, height)
        light = main_light() if light is None else np.asarray(light, np.float32)
        c2w = np.asarray(c2w, np.float32)
        if self._c2w is None or not np.array_equal(self._c2w, c2w):   # transform.hasChanged (:44-47)
            self.currentSample = 0
            self._c2w = c2w.copy()
        c = column_major(c2w)
        p = column_major(inv_proj)
        lt = np.ascontiguousarray(light, np.float32)
        check(_lib.lib().svo_set_camera(self._ctx, c.ctypes.data, p.ctypes.data, float(pixel_offset[0]),
                                        float(pixel_offset[1]), lt.ctypes.data), "svo_set_camera")
        self._camera_set = True

    def _set_option(self, bit, enable):
        self._options = (self._options | bit) if enable else (self._options & ~bit)
        check(_lib.lib().svo_set_options(self._ctx, self._options), "svo_set_options")

    def SetShadowRays(self, enable=True):
        """Trace one shadow ray per primary hit toward -_DirectionalLight (the
        reference's commented-out test, RaytraceCompute.compute:105-112)."""
        self._set_option(_lib.SVO_OPT_SHADOW_RAYS, enable)

    def set_count_beam(self, enable=True):
        """SVO_OPT_COUNT_BEAM: count_fetches_device counts the fetches of the walk the render runs
        (from the beam start) instead of the reference's walk from the cube entry."""
        self._set_option(_lib.SVO_OPT_COUNT_BEAM, enable)

    def set_kernel_timing(self, enable=True):
        """Bracket the primary-ray kernel of every launch with HIP events
        (measurement only; read with kernel_time())."""
        self._set_option(_lib.SVO_OPT_KERNEL_TIMING, enable)

    def kernel_time(self):
        """(mean primary-kernel ms, launches) over the launches timed since the last call."""
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        check(_lib.lib().svo_kernel_time(self._ctx, ctypes.byref(ms), ctypes.byref(n)), "svo_kernel_time")
        return ms.value, n.value

    def stage_time(self, stage):
        """(mean ms, launches) of a timed stage: _lib.STAGE_KERNEL or STAGE_ASSEMBLE."""
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        check(_lib.lib().svo_stage_time(self._ctx, int(stage), ctypes.byref(ms), ctypes.byref(n)), "svo_stage_time")
        return ms.value, n.value

    def stage_times(self, stage=_lib.STAGE_KERNEL, cap=1 << 16):
        """Every timed launch's duration (ms, float32 array in launch order) of a stage
        since the last read (svo_stage_times)."""
        out = np.zeros(cap, np.float32)
        n = ctypes.c_size_t()
        check(_lib.lib().svo_stage_times(self._ctx, int(stage), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                         cap, ctypes.byref(n)), "svo_stage_times")
        return out[:min(n.value, cap)].copy()

    def set_band_deal(self, owner=None):
        """Multi-device context: deal band b to member owner[b % len(owner)]
        (distributed.weighted_owner gives fewer bands to devices[0]); None =
        round-robin."""
        n = 0 if owner is None else len(owner)
        arr = (ctypes.c_uint8 * max(n, 1))(*([int(o) for o in owner] if owner else [0]))
        check(_lib.lib().svo_set_band_deal(self._ctx, n, arr if n else None), "svo_set_band_deal")

    def num_devices(self):
        n = ctypes.c_int()
        check(_lib.lib().svo_num_devices(self._ctx, ctypes.byref(n)), "svo_num_devices")
        return n.value

    def member_links(self):
        """[(device, link name)] per member: how each member's band payload reaches the
        display device (svo_get_member_link: "self", "xgmi_peer_pull" or "peer_copy")."""
        out = []
        for i in range(self.num_devices()):
            d, k = ctypes.c_int(), ctypes.c_int()
            check(_lib.lib().svo_get_member_link(self._ctx, i, ctypes.byref(d), ctypes.byref(k)),
                  "svo_get_member_link")
            out.append((d.value, _lib.LINK_NAMES.get(k.value, str(k.value))))
        return out

    def member(self, index):
        """The per-device context `index` (owned by this one) as a RaytracingMaster view."""
        c = ctypes.c_void_p()
        check(_lib.lib().svo_get_member(self._ctx, int(index), ctypes.byref(c)), "svo_get_member")
        return _MemberView(self, c)

    # ----------------------------------------------------------------- render
    def Render(self, width, height, stack_mode=STACK_HLSL, want_rgba=True, want_hits=True, out=None):
        """Blocking render into host arrays: (rgba[H, W, 4] float32, hits[H, W] svo_hit).
        out: an earlier call's (rgba, hits) to write again (a render loop's reused arrays; fresh
        arrays pay the first-touch page faults of 83 MB per 1080p frame)."""
        if out is not None:
            rgba, hits = out
            assert rgba is None or (rgba.dtype == np.float32 and rgba.size == height * width * 4 and rgba.flags.c_contiguous)
            assert hits is None or (hits.dtype == HIT_DTYPE and hits.size == height * width and hits.flags.c_contiguous)
        else:
            rgba = np.zeros((height, width, 4), np.float32) if want_rgba else None
            hits = np.zeros((height, width), HIT_DTYPE) if want_hits else None
        check(_lib.lib().svo_render(self._ctx, width, height, stack_mode,
                                    None if rgba is None else rgba.ctypes.data,
                                    None if hits is None else hits.ctypes.data), "svo_render")
        return rgba, hits

    def RenderProgressive(self, width, height, stack_mode=STACK_HLSL, want_rgba8=True, want_rgba=False):
        """OnRenderImage end to end (RaytracingMaster.cs:55-74): render a sample at
        the current camera, blend it into the plugin's device-resident accumulation
        frame with _Sample = currentSample (AddShader), then currentSample += 1.
        Returns (rgba8[H, W] uint32 display words or None, rgba[H, W, 4] float32
        accumulated frame or None); only those cross PCIe."""
        rgba8 = np.zeros((height, width), np.uint32) if want_rgba8 else None
        rgba = np.zeros((height, width, 4), np.float32) if want_rgba else None
        if getattr(self, "_accum_size", None) != (width, height):
            # a new render-target size (InitRenderTexture, RaytracingMaster.cs:76-88): the
            # plugin starts a fresh accumulation frame, so the sample count restarts too
            self._accum_size = (width, height)
            self.currentSample = 0
        check(_lib.lib().svo_render_progressive(self._ctx, width, height, stack_mode, self.currentSample,
                                                None if rgba8 is None else rgba8.ctypes.data,
                                                None if rgba is None else rgba.ctypes.data),
              "svo_render_progressive")
        self.currentSample += 1
        return rgba8, rgba

    def RenderProgressiveAsync(self, width, height, stack_mode=STACK_HLSL, copy=True, rgb=False):
        """OnRenderImage through the pipelined readback (svo_render_progressive_async):
        enqueue this sample and return the PREVIOUS frame's display pixels (rgba8[H, W]
        uint32 words, or with rgb=True uint8[H, W, 3]; None on the first call at a size or
        format).  copy=False returns a view of the plugin's pinned buffer, valid until the
        call after next."""
        if getattr(self, "_accum_size", None) != (width, height):
            self._accum_size = (width, height)
            self.currentSample = 0
        ptr = ctypes.c_void_p()
        fmt = _lib.PIXELS_RGB8 if rgb else _lib.PIXELS_RGBA8
        check(_lib.lib().svo_render_progressive_async(self._ctx, width, height, stack_mode, self.currentSample, fmt,
                                                      ctypes.byref(ptr)), "svo_render_progressive_async")
        self.currentSample += 1
        self._pin_rgb = rgb
        return self._pinned_frame(ptr, width, height, copy, rgb)

    def ProgressiveLast(self, width, height, copy=True):
        """The most recent frame of RenderProgressiveAsync (waits for its copy)."""
        ptr = ctypes.c_void_p()
        check(_lib.lib().svo_progressive_last(self._ctx, ctypes.byref(ptr)), "svo_progressive_last")
        return self._pinned_frame(ptr, width, height, copy, getattr(self, "_pin_rgb", False))

    @staticmethod
    def _pinned_frame(ptr, width, height, copy, rgb=False):
        if not ptr.value:
            return None
        if rgb:
            a = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(height, width, 3))
        else:
            a = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint32)), shape=(height, width))
        return a.copy() if copy else a

    def render_device(self, width, height, rgba_ptr=None, hits_ptr=None, stack_mode=STACK_HLSL,
                      band=None, stream=None):
        """Asynchronous render into device buffers (raw device pointers, e.g. torch
        tensor.data_ptr()), optionally only this rank's row bands."""
        b = None if band is None else ctypes.byref(make_band(band))
        check(_lib.lib().svo_render_device(self._ctx, width, height, stack_mode, b, rgba_ptr, hits_ptr, stream),
              "svo_render_device")

    def render_frame(self, width, height, hits=None, rgba=None, rgba8=None, compact=None, position=None,
                     voxel=None, layout=LAYOUT_BAND, stack_mode=STACK_HLSL, band=None, stream=None, rgb8=None,
                     hitmask=None):
        """Asynchronous render of every requested output (device pointers).
        layout LAYOUT_BAND: buffers hold only `band`'s rows; LAYOUT_FRAME: full-frame
        buffers.  A multi-device context renders the whole frame (band None) onto
        devices[0]."""
        # band: a (rows, rank, count[, owner]) tuple or a prebuilt _lib.SvoBand (per-frame callers
        # build it once: the owner table costs host time on every call otherwise)
        b = None if band is None else ctypes.byref(band if isinstance(band, _lib.SvoBand) else make_band(band))
        f = _frame(hits, rgba, rgba8, compact, position, voxel, layout, rgb8, hitmask)
        check(_lib.lib().svo_render_frame(self._ctx, width, height, stack_mode, b, ctypes.byref(f), stream),
              "svo_render_frame")

    def render_samples(self, width, height, offsets, first_sample, accum, rgba8=None, rgb8=None, layout=LAYOUT_BAND,
                       stack_mode=STACK_HLSL, band=None, stream=None):
        """Samples in flight (svo_render_samples): trace len(offsets) jittered samples
        (offsets: [S, 2] pixel offsets, S <= 8) in one launch and blend them in order into
        the device RGBA32F frame `accum` as _Sample = first_sample + k; rgba8 / rgb8 (device
        pointers, nullable): the blended frame's display words / 3-byte RGB."""
        off = np.ascontiguousarray(offsets, np.float32).reshape(-1, 2)
        b = None if band is None else ctypes.byref(band if isinstance(band, _lib.SvoBand) else make_band(band))
        check(_lib.lib().svo_render_samples(self._ctx, width, height, stack_mode, b, len(off),
                                            off.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), int(first_sample),
                                            accum, rgba8, rgb8, layout, stream), "svo_render_samples")

    def assemble_frame(self, width, height, parts, part_format, band_rows=None, hits=None, rgba=None, rgba8=None,
                       compact=None, skip_part=-1, stream=None, owner=None, deal=None):
        """Rebuild a frame (full-frame device buffers) from band parts: parts[m] = the
        device pointer of rank m's band payload (compact records or RGBA8 words).
        The deal: band_rows-row bands, round-robin, or owner[b % len(owner)] = the
        part holding band b (weighted deal)."""
        # parts may be a prebuilt ctypes array and deal a prebuilt _lib.SvoBand (per-frame callers)
        arr = parts if isinstance(parts, ctypes.Array) else (ctypes.c_void_p * len(parts))(*[p if p else None for p in parts])
        f = _frame(hits, rgba, rgba8, compact, None, None, LAYOUT_FRAME)
        rows = self.band_rows if band_rows is None else band_rows
        if deal is None:
            deal = make_band((rows, 0, len(parts)) if owner is None else (rows, 0, len(parts), owner))
        check(_lib.lib().svo_assemble_frame(self._ctx, width, height, ctypes.byref(deal), len(parts), arr,
                                            part_format, skip_part, ctypes.byref(f), stream),
              "svo_assemble_frame")

    def pack_hits(self, width, height, band, rgb8, part, stream=None):
        """Sparse band payload (svo_rt.h layout): `part` (device pointer, capacity
        _lib.sparse_part_bytes) starts with the band's hit masks
        (render_frame(hitmask=part)); write the tile offsets and the hit count
        behind them and pack the RGB of the hit pixels from the band's dense
        `rgb8` after that."""
        band = band if band is not None else (self.band_rows, 0, 1)
        b = ctypes.byref(band if isinstance(band, _lib.SvoBand) else make_band(band))
        check(_lib.lib().svo_pack_hits(self._ctx, width, height, b, rgb8, part, stream), "svo_pack_hits")

    def beam_starts_device(self, width, height, starts_ptr, band=None, stream=None):
        """svo_beam_starts: every primary ray's beam start (SVO-space t, -inf: the cube entry) into a
        device float buffer of the band's pixels (diagnostics)."""
        b = None if band is None else ctypes.byref(make_band(band))
        check(_lib.lib().svo_beam_starts(self._ctx, width, height, b, starts_ptr, stream), "svo_beam_starts")

    def count_fetches_device(self, width, height, fetch_ptr, stack_mode=STACK_HLSL, band=None, stream=None):
        b = None if band is None else ctypes.byref(make_band(band))
        check(_lib.lib().svo_count_fetches(self._ctx, width, height, stack_mode, b, fetch_ptr, stream),
              "svo_count_fetches")

    def accumulate_device(self, accum_ptr, sample_ptr, n_px, sample=None, stream=None):
        """Blend one RGBA32F sample frame into the accumulation frame (device
        pointers) with _Sample = `sample` (default: currentSample, which then
        advances like _currentSample++ after the Blit)."""
        n = self.currentSample if sample is None else int(sample)
        check(_lib.lib().svo_accumulate(self._ctx, accum_ptr, sample_ptr, int(n_px), n, stream), "svo_accumulate")
        if sample is None:
            self.currentSample += 1

    def forget_stream(self, stream):
        """svo_forget_stream: the caller is about to destroy `stream` (a hipStream_t handle)."""
        check(_lib.lib().svo_forget_stream(self._ctx, stream), "svo_forget_stream")

    def synchronize(self):
        check(_lib.lib().svo_synchronize(self._ctx), "svo_synchronize")

    def info(self):
        n = ctypes.c_size_t()
        d = ctypes.c_int()
        dev = ctypes.c_int()
        check(_lib.lib().svo_get_info(self._ctx, ctypes.byref(n), ctypes.byref(d), ctypes.byref(dev)),
              "svo_get_info")
        return {"n_nodes": n.value, "depth": d.value, "device": dev.value}

    def close(self):
        if self._ctx:
            _lib.lib().svo_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _MemberView(RaytracingMaster):
    """One device of a multi-device context: queries and device renders on that
    device alone (not destroyed on its own)."""

    def __init__(self, owner, ctx):   # noqa: D107 -- no svo_create: the group owns the context
        self._owner = owner
        self._ctx = ctx
        self._options = owner._options
        self._config = dict(owner._config)
        self.currentSample = 0
        self._c2w = None
        self.devices = None
        self.band_rows = owner.band_rows
        self.device = self.info()["device"]

    def close(self):
        self._ctx = ctypes.c_void_p()


def band_rows(height, band):
    """Global row indices owned by `band` = (band_rows, band_rank, band_count) (round-robin)
    or (band_rows, band_rank, band_count, owner) (band b belongs to owner[b % len(owner)]),
    in order."""
    rows, rank, count = band[:3]
    ys = np.arange(height)
    if len(band) == 3:
        return ys[(ys // rows) % count == rank]
    owner = np.asarray(band[3], np.int64)
    return ys[owner[(ys // rows) % len(owner)] == rank]


__all__ = ["RaytracingMaster", "SVOData", "SvoError", "STACK_HLSL", "STACK_EXACT", "HIT_DTYPE", "band_rows"]
