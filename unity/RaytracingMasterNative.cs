// RaytracingMasterNative.cs -- Unity-side drop-in for Assets/Scripts/SVO/GPU/RaytracingMaster.cs
// that drives the MI355X plugin (libsvo_rt.so, include/svo_rt.h) through P/Invoke instead of
// ComputeShader.Dispatch.  NOT compiled in this repository (no C# toolchain in the build image);
// it is the binding a Unity maintainer adds next to the reference script (see INTEGRATION.md).
using System;
using System.Runtime.InteropServices;
using UnityEngine;

public static class SvoNative {
    const string Lib = "svo_rt";        // libsvo_rt.so in Assets/Plugins/x86_64
    const string Builder = "svo_build"; // libsvo_build.so: the native NaiveCreator (include/svo_build.h)
    public const int StackHlsl = 0, StackExact = 1;

    [StructLayout(LayoutKind.Sequential)]
    public struct SvoHit { public uint parent; public byte hitIdx; public byte hitScale; public ushort flags;
                           public float t, nx, ny, nz; }                          // 24 bytes == svo_hit

    [DllImport(Lib)] public static extern int svo_create(int device, UIntPtr capacityNodes, out IntPtr ctx);
    [DllImport(Lib)] public static extern int svo_create_multi(int[] devices, int numDevices, UIntPtr capacityNodes,
                                                               int bandRows, out IntPtr ctx);
    [DllImport(Lib)] public static extern int svo_set_buffer(IntPtr ctx, int[] desc, UIntPtr nDesc,
                                                             uint[] att, UIntPtr nAtt, UIntPtr dstOffset);
    // wide node format (svo_rt.h): first_child_abs << 32 | valid << 8 | nonleaf -- any pool the builder makes,
    // straight from the builder's native arrays (no managed copy)
    [DllImport(Lib)] public static extern int svo_set_buffer_v2(IntPtr ctx, IntPtr nodes, UIntPtr nNodes,
                                                                IntPtr att, UIntPtr nAtt, UIntPtr dstOffset);
    [DllImport(Lib)] public static extern int svo_get_info(IntPtr ctx, out UIntPtr nNodes, out int maxDepth,
                                                           out int device);
    [DllImport(Lib)] public static extern int svo_set_camera(IntPtr ctx, float[] c2w, float[] invProj,
                                                             float pxOffX, float pxOffY, float[] light);
    [DllImport(Lib)] public static extern int svo_render(IntPtr ctx, int width, int height, int stackMode,
                                                         float[] rgbaOut, [Out] SvoHit[] hitsOut);
    [DllImport(Lib)] public static extern int svo_render_progressive(IntPtr ctx, int width, int height, int stackMode,
                                                                     uint sample, [Out] uint[] rgba8Out,
                                                                     [Out] float[] rgbaOut);
    // pipelined readback: returns the previous frame's RGBA8 words in plugin-owned pinned memory
    // (valid until the call after next), the D2H of this frame overlapping the next render
    public const int PixelsRgba8 = 0, PixelsRgb8 = 1;   // TextureFormat.RGBA32 / RGB24
    [DllImport(Lib)] public static extern int svo_render_progressive_async(IntPtr ctx, int width, int height,
                                                                           int stackMode, uint sample, int pixelFormat,
                                                                           out IntPtr frame);
    [DllImport(Lib)] public static extern int svo_destroy(IntPtr ctx);
    [DllImport(Lib)] public static extern IntPtr svo_last_error();

    // svo_config (include/svo_rt.h, ABI 10): the render policy, versioned by size -- field order and
    // types exactly the header's (132 bytes; tests/test_boundary.py checks the C layout)
    [StructLayout(LayoutKind.Sequential)]
    public struct SvoConfig {
        public uint size, version;
        public int tileOrder, xcdStrips, issuePriority, orderEvery, moveEvery, moveSpread, relayout, fetchAll,
                   loopForm;
        public float latRatio;
        public int segments;
        public uint segTableLatency, segTableIssue, segTableThin;
        public float segRatio, segThinRatio;
        public int segCap, segMinChain, segMove, segJitter, segAll;
        public uint segScramble;
        public int beam, beamBack, shadowForm, shadowOrder, readback, hostCopyThreads, sparsePayload, peerCopy;
        public int beamBackHeld;   // config version 2
    }
    [DllImport(Lib)] public static extern int svo_get_config(IntPtr ctx, ref SvoConfig cfg);
    [DllImport(Lib)] public static extern int svo_set_config(IntPtr ctx, ref SvoConfig cfg);

    [StructLayout(LayoutKind.Sequential)]
    public struct SvobResult {   // == svob_result
        public UIntPtr nNodes; public int depth; public int v1Ok;
        public IntPtr descriptors, nodes, attachments; public UIntPtr nLeaves;
    }
    [DllImport(Builder)] public static extern int svob_build_sampler(int device, int sampler, int maxLevel,
                                                                     out SvobResult result);
    [DllImport(Builder)] public static extern void svob_free(ref SvobResult result);
    [DllImport(Builder)] public static extern IntPtr svob_last_error();

    public static void Check(int rc, string what) {
        if (rc != 0) throw new InvalidOperationException(what + ": " + Marshal.PtrToStringAnsi(svo_last_error()));
    }
    public static void CheckBuild(int rc, string what) {
        if (rc != 0) throw new InvalidOperationException(what + ": " + Marshal.PtrToStringAnsi(svob_last_error()));
    }

    // The HLSL float2 stack (NVIDIASVO.compute:98) rounds parent indices above 2^24 nodes
    // (SURVEY.md Appendix A): such pools (C4, C5) trace with the exact stack
    public static int StackModeFor(IntPtr ctx) {
        Check(svo_get_info(ctx, out UIntPtr n, out int depth, out int device), "svo_get_info");
        return (ulong)n > (1UL << 24) ? StackExact : StackHlsl;
    }

    // Unity Matrix4x4 is column-major in memory (m00, m10, m20, m30, m01, ...), which is the C-ABI order.
    public static float[] ToArray(Matrix4x4 m) {
        var a = new float[16];
        for (int i = 0; i < 16; i++) a[i] = m[i];   // Matrix4x4 indexer is column-major
        return a;
    }
}

public class RaytracingMasterNative : MonoBehaviour {
    public Light DirectionalLight;
    // the reference's [Range(1, 8)] (RaytracingMaster.cs:16-17) is widened: the native builder
    // makes the BASELINE pools up to 8192^3 (maxLevel 14) in seconds
    [Range(1, 14)] public int maxLevel = 5;
    public SampleFunctions.Type sampleType = SampleFunctions.Type.Custom1;
    [Range(1, 8)] public int gpus = 1;   // > 1: the frame is split in 8-row bands over GPUs 0..gpus-1

    // Render policy (svo_config): the Inspector fields a developer tunes; the defaults are the
    // library's (svo_get_config(NULL)).  None changes the image -- only where the time goes.
    [Header("Render policy (svo_config)")]
    public bool beamStarts = true;               // beam: rays start at their tile's lower bound of the hit t
    [Range(0, 8)] public int beamBack = 2;       // a new view's splat: boxes this many levels above the leaves
    [Range(-1, 8)] public int beamBackHeld = 0;  // a held view's finer re-splat (-1: beamBack)
    public bool segmentedRays = true;            // segments: heavy tiles traced as exact t-segments
    public bool costOrderedDispatch = true;      // tile_order: heaviest tiles dispatched first
    [Range(1, 32)] public int moveEvery = 4;     // while the camera moves, rebuild the order every k-th frame
    public enum ShadowForm { Fused = 0, TilePass = 1, CompactedList = 2 }
    public ShadowForm shadowForm = ShadowForm.Fused;

    IntPtr _ctx;
    Camera _camera;
    Texture2D _frame;
    uint[] _rgba8;
    uint _currentSample = 0;   // RaytracingMaster.cs:12
    int _stackMode = SvoNative.StackHlsl;   // chosen from the uploaded pool (SvoNative.StackModeFor)

    void Awake() {
        _camera = GetComponent<Camera>();
        InitializeSVOBuffer();
    }

    // RaytracingMaster.cs:44-53: a moved camera restarts the accumulation; key R rebuilds the SVO
    void Update() {
        if (transform.hasChanged) {
            _currentSample = 0;
            transform.hasChanged = false;
        }
        if (Input.GetKeyDown(KeyCode.R)) SetSVOBuffer();
    }

    // RaytracingMaster.cs:111-116
    public void InitializeSVOBuffer() {
        CreateContext((UIntPtr)(1073741824 / 8));
    }

    void CreateContext(UIntPtr capacity) {
        IntPtr ctx;
        if (gpus <= 1) {
            SvoNative.Check(SvoNative.svo_create(0, capacity, out ctx), "svo_create");
        } else {   // one SVO replica per GPU, bands gathered to GPU 0 over xGMI; every other call is unchanged
            var devices = new int[gpus];
            for (int i = 0; i < gpus; i++) devices[i] = i;
            SvoNative.Check(SvoNative.svo_create_multi(devices, gpus, capacity, 8, out ctx), "svo_create_multi");
        }
        _ctx = ctx;
        ApplyConfig();
    }

    // the Inspector fields into the context's svo_config; the other fields keep the library's values
    void ApplyConfig() {
        if (_ctx == IntPtr.Zero) return;
        var cfg = new SvoNative.SvoConfig { size = (uint)Marshal.SizeOf<SvoNative.SvoConfig>() };
        SvoNative.Check(SvoNative.svo_get_config(_ctx, ref cfg), "svo_get_config");
        cfg.beam = beamStarts ? 1 : 0;
        cfg.beamBack = beamBack;
        cfg.beamBackHeld = beamBackHeld;
        cfg.segments = segmentedRays ? 1 : 0;
        cfg.tileOrder = costOrderedDispatch ? 1 : 0;
        cfg.moveEvery = moveEvery;
        cfg.shadowForm = (int)shadowForm;
        SvoNative.Check(SvoNative.svo_set_config(_ctx, ref cfg), "svo_set_config");
    }

    void OnValidate() { ApplyConfig(); }   // an Inspector edit at run time takes effect at the next frame

    // RaytracingMaster.cs:90-109 (key R): NaiveCreator.Create(SampleFunctions.functions[sampleType], maxLevel)
    // by the native builder on GPU 0, uploaded in the wide node format -- every BASELINE pool from
    // 256^3 up has child pointers beyond the reference's 16 bits.  The pool replaces the old one (the
    // capacity is the 1 GiB of InitializeSVOBuffer; a bigger pool gets a context of its size).
    void SetSVOBuffer() {
        // SampleFunctions.functions[5] (Custom2) is null in the reference (SampleFunctions.cs:13-48):
        // its key R would throw there too; say so instead of calling the builder
        if ((int)sampleType > (int)SampleFunctions.Type.Custom1) {
            Debug.LogError("sampleType " + sampleType + " has no sampler in the reference (SampleFunctions.functions)");
            return;
        }
        SvoNative.CheckBuild(SvoNative.svob_build_sampler(0, (int)sampleType, maxLevel, out var r), "svob_build_sampler");
        try {
            ulong n = (ulong)r.nNodes;
            if (n > (ulong)(1073741824 / 8)) {   // beyond InitializeSVOBuffer's capacity
                SvoNative.svo_destroy(_ctx);
                _ctx = IntPtr.Zero;                // never left pointing at the freed context
                CreateContext((UIntPtr)n);         // assigns _ctx only once the new context exists
            }
            SvoNative.Check(SvoNative.svo_set_buffer_v2(_ctx, r.nodes, r.nNodes, r.attachments, (UIntPtr)(2 * n),
                                                        UIntPtr.Zero), "svo_set_buffer_v2");
        } finally {
            SvoNative.svob_free(ref r);
        }
        _stackMode = SvoNative.StackModeFor(_ctx);
        _currentSample = 0;
    }

    // RaytracingMaster.cs:118-135 (attachments land at 2*offset: the reference's offset bug is fixed)
    public void SetSVOBuffer(RT.SVOData data, int offset = 0) {
        var desc = data.childDescriptors.ToArray();
        var att = data.attachments.ToArray();
        SvoNative.Check(SvoNative.svo_set_buffer(_ctx, desc, (UIntPtr)desc.Length, att, (UIntPtr)att.Length,
                                                 (UIntPtr)offset), "svo_set_buffer");
        _stackMode = SvoNative.StackModeFor(_ctx);
    }

    // RaytracingMaster.cs:32-41 + 55-74: the sample is rendered, blended into the plugin's
    // device-resident accumulation frame with _Sample = _currentSample (AddShader.shader:44-47),
    // and only the accumulated display frame (RGBA8, 4 B/px) crosses PCIe -- into the plugin's
    // pinned buffer, on a copy stream, while the next frame renders: the call returns the
    // PREVIOUS frame's words, which LoadRawTextureData copies straight from that pointer (no
    // managed array).  One frame of display latency; pipelined = false uses the blocking call.
    public bool pipelined = true;

    void OnRenderImage(RenderTexture source, RenderTexture destination) {
        Vector3 l = DirectionalLight.transform.forward;
        SvoNative.Check(SvoNative.svo_set_camera(_ctx, SvoNative.ToArray(_camera.cameraToWorldMatrix),
                                                 SvoNative.ToArray(_camera.projectionMatrix.inverse),
                                                 UnityEngine.Random.value, UnityEngine.Random.value,
                                                 new[] { l.x, l.y, l.z, DirectionalLight.intensity }), "svo_set_camera");
        int w = Screen.width, h = Screen.height;
        // the pipelined path moves 3-byte pixels (RGB24: a quarter fewer bytes over PCIe); `pipelined`
        // is an Inspector field, so a toggle at run time recreates the texture in the other format
        TextureFormat want = pipelined ? TextureFormat.RGB24 : TextureFormat.RGBA32;
        if (_frame == null || _frame.width != w || _frame.height != h || _frame.format != want) {
            _frame = new Texture2D(w, h, want, false, true);
            _rgba8 = new uint[w * h];
            _currentSample = 0;   // a new render target: the plugin starts a fresh accumulation frame
        }
        if (pipelined) {
            SvoNative.Check(SvoNative.svo_render_progressive_async(_ctx, w, h, _stackMode, _currentSample,
                                                                   SvoNative.PixelsRgb8, out IntPtr prev),
                            "svo_render_progressive_async");
            if (prev != IntPtr.Zero) {   // NULL only on the first frame at this size
                _frame.LoadRawTextureData(prev, w * h * 3);
                _frame.Apply(false);
            }
        } else {
            SvoNative.Check(SvoNative.svo_render_progressive(_ctx, w, h, _stackMode, _currentSample, _rgba8, null),
                            "svo_render_progressive");
            _frame.SetPixelData(_rgba8, 0);
            _frame.Apply(false);
        }
        Graphics.Blit(_frame, destination);   // already accumulated: a plain copy, no AddMaterial
        _currentSample++;
    }

    void OnDestroy() {
        if (_ctx != IntPtr.Zero) SvoNative.svo_destroy(_ctx);
    }
}
