// TrueTraceHip.cs — P/Invoke binding a TrueTrace maintainer adds to call the MI355X engine
// (libtruetrace_hip.so, include/truetrace_hip.h) in place of the kernel_trace dispatch.
//
// Style follows the reference's only native-plugin boundary,
// TrueTrace/Resources/Utility/UnityDenoiserPlugin/UnityDenoiserPlugin.cs:14-85: blittable
// [StructLayout(Sequential)] structs, an IntPtr handle owned by an IDisposable wrapper.
// Not compiled in this repository (no .NET toolchain in the build image); the struct layouts are
// checked against the C header by tests/test_abi.py through the Python mirror of the same ABI.
using System;
using System.Runtime.InteropServices;

namespace TrueTrace.Hip
{
    public enum TTStatus : int
    {
        Ok = 0, InvalidArg = 1, OutOfMemory = 2, Hip = 3, Unsupported = 4, StackOverflow = 5, NoDevice = 6, NoScene = 7
    }

    [Flags]
    public enum TTTraceFlags : uint
    {
        None = 0, DevicePtrs = 1u << 0, UseReSTIRGI = 1u << 1, UseASVGF = 1u << 2, Stats = 1u << 3, Async = 1u << 4,
        IgnoreGlass = 1u << 5,       // IgnoreGlassMain  (IntersectionKernels.compute:42-44)
        IgnoreBackfacing = 1u << 6,  // IgnoreBackfacing (IntersectionKernels.compute:45-47)
        AdaptiveOrder = 1u << 7,     // dequeue the previous launch's costliest 8x8 tiles first (same results)
        RadianceCache = 1u << 7,     // tt_trace_shadow_ex: the RadianceCache define (GlobalDefines.cginc:15)
        VisibilityCheck = 1u << 8    // tt_trace_shadow_ex: VisabilityCheckCompute (CommonData.cginc:710-819)
    }

    [StructLayout(LayoutKind.Sequential)]
    public struct TTConfig
    {
        public int device;
        public uint flags;
        public ulong maxRays;
        public IntPtr stream;
    }

    [StructLayout(LayoutKind.Sequential)]
    public struct TTTraceParams
    {
        public uint nRays;        // BufferSizes[CurBounce].tracerays
        public int bounce;        // CurBounce
        public float farPlane;    // FarPlane
        public uint screenWidth;
        public uint screenHeight;
        public TTTraceFlags flags;
    }

    [StructLayout(LayoutKind.Sequential)]
    public struct TTStats
    {
        public ulong rays, nodeVisits, triTests, blasEntries, hits, repsExhausted, stackOverflows, accepts;
        public float kernelMs;
        public uint pad;
    }

    [StructLayout(LayoutKind.Sequential)]
    public struct TTShadowParams
    {
        public uint nRays;        // BufferSizes[CurBounce].shadow_rays
        public int bounce;        // CurBounce
        public uint screenWidth;
        public uint screenHeight;
        public TTTraceFlags flags;
    }

    [StructLayout(LayoutKind.Sequential)]
    public unsafe struct TTBlasRefitParams
    {
        public uint meshIndex;     // _MeshData record: TriOffset, NodeOffset, BLAS root
        public uint nTris;
        public uint nVertices;
        public uint vertexStride;  // VertexBuffer stride / 4; position at +0, normal at +3
        public fixed float transform[16];
        public uint flags;
    }

    /// Generate's camera (RayGenKernels.compute:40-57): Unity's cameraToWorldMatrix and projectionMatrix.inverse,
    /// column-major (the memory order of UnityEngine.Matrix4x4).
    [StructLayout(LayoutKind.Sequential)]
    public unsafe struct TTCamera
    {
        public fixed float camToWorld[16];
        public fixed float camInvProj[16];
        public float nearPlane, farPlane;
        public uint width, height;
        public int jitter;             // 1: the !UseReCur sub-pixel jitter
        public int framesAccumulated;  // random() seed input
        public int maxBounce;
        public TTTraceFlags flags;     // DevicePtrs [| Async]
    }

    [Flags]
    public enum TTGroupFlags : uint { None = 0, CopyGather = 1u << 0, Bounce = 1u << 1, Info = 1u << 2 }

    /// tt_group_config: the screen a multi-GPU group traces, its tile edge, frames in flight and flags.
    [StructLayout(LayoutKind.Sequential)]
    public struct TTGroupConfig
    {
        public uint width, height;
        public uint tile;      // 0: 64
        public uint slots;     // 0: 2
        public TTGroupFlags flags;
        public uint batch;     // frames per call (0: 1): frames_accumulated + b, b < batch, as one B-frames-tall screen
    }

    /// Column-major 4x4 (the memory order of UnityEngine.Matrix4x4: m00, m10, m20, m30, m01, ...).
    public struct Matrix4x4Floats { public float[] m; }

    public static class Native
    {
        const string Lib = "truetrace_hip";
        [DllImport(Lib)] public static extern int tt_abi_version();
        [DllImport(Lib)] public static extern TTStatus tt_ctx_create(ref TTConfig cfg, out IntPtr ctx);
        [DllImport(Lib)] public static extern TTStatus tt_ctx_destroy(IntPtr ctx);
        [DllImport(Lib)] public static extern IntPtr tt_last_error(IntPtr ctx);
        [DllImport(Lib)] public static extern int tt_device_count();
        [DllImport(Lib)] public static extern TTStatus tt_stream_create(int device, out TTStreamHandle stream);
        [DllImport(Lib)] public static extern TTStatus tt_stream_destroy(IntPtr stream);
        [DllImport(Lib)] public static extern uint tt_stream_live_count();
        // every library stream still alive, synchronised and destroyed: OnApplicationQuit / AppDomain.DomainUnload
        [DllImport(Lib)] public static extern TTStatus tt_shutdown();
        // Element types are the reference's own host structs: BVHNode8DataCompressed (80 B),
        // CudaTriangle (88 B), int, MyMeshDataCompacted (88 B), MaterialData (252 B).
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_upload(IntPtr ctx,
            void* nodes, uint nNodes, void* tris, uint nTris, int* tlasIndices, uint nTlas,
            void* meshData, uint nMesh, void* materials, uint nMat);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_update_nodes(IntPtr ctx, uint first, uint count, void* nodes);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_update_meshdata(IntPtr ctx, uint first, uint count, void* meshData);
        // GlobalRays (RayData, 48 B, hits written in place), _PrimaryTriangleInfo (uint4 per pixel),
        // GlobalColors (ColData, 64 B).
        [DllImport(Lib)] public static extern unsafe TTStatus tt_trace_closest(IntPtr ctx, ref TTTraceParams p,
            void* globalRays, uint* primaryInfo, void* globalColors, out TTStats stats);
        // ShadowRayData (48 B, t = 0 written for occluded rays), float4 visibility per ray,
        // GlobalColors (ColData, 64 B), NEEPosA (float4 per pixel); the last three nullable.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_trace_shadow(IntPtr ctx, ref TTShadowParams p,
            void* shadowRays, float* visibility, void* globalColors, float* neePos, out TTStats stats);
        // + CacheBuffer (PropogatedCacheData, 48 B per pixel, nullable): the full :457-485 output contract.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_trace_shadow_ex(IntPtr ctx, ref TTShadowParams p,
            void* shadowRays, float* visibility, void* globalColors, float* neePos, void* cacheBuffer, out TTStats stats);
        // Device-pointer forms: the same entry points, the buffers passed as HIP device addresses.
        [DllImport(Lib, EntryPoint = "tt_trace_closest")] public static extern TTStatus tt_trace_closest_dev(IntPtr ctx,
            ref TTTraceParams p, IntPtr globalRays, IntPtr primaryInfo, IntPtr globalColors, out TTStats stats);
        [DllImport(Lib, EntryPoint = "tt_trace_shadow_ex")] public static extern TTStatus tt_trace_shadow_dev(IntPtr ctx,
            ref TTShadowParams p, IntPtr shadowRays, IntPtr visibility, IntPtr globalColors, IntPtr neePos,
            IntPtr cacheBuffer, out TTStats stats);
        // Indirect dispatch (BufferSizes[CurBounce].tracerays / .shadow_rays kept on the GPU, the reference's
        // TransferKernel + DispatchIndirect): traces min(*nRaysDev, p.nRays) rays; device pointers, async.
        [DllImport(Lib)] public static extern TTStatus tt_trace_closest_indirect(IntPtr ctx, ref TTTraceParams p,
            IntPtr nRaysDev, IntPtr globalRays, IntPtr primaryInfo, IntPtr globalColors);
        [DllImport(Lib)] public static extern TTStatus tt_trace_shadow_ex_indirect(IntPtr ctx, ref TTShadowParams p,
            IntPtr nRaysDev, IntPtr shadowRays, IntPtr visibility, IntPtr globalColors, IntPtr neePos, IntPtr cacheBuffer);
        // tt_trace_closest + each ray's 16-B hit record written contiguously to hitsOut (the multi-GPU gather's input)
        [DllImport(Lib)] public static extern TTStatus tt_trace_closest_hits(IntPtr ctx, ref TTTraceParams p,
            IntPtr globalRays, IntPtr primaryInfo, IntPtr globalColors, IntPtr hitsOut);
        // dst traces src's scene buffers (no copy) on its own stream: the parts of a frame share one scene
        [DllImport(Lib)] public static extern TTStatus tt_ctx_share_scene(IntPtr dst, IntPtr src);
        [DllImport(Lib)] public static extern TTStatus tt_ctx_share_blas(IntPtr dst, IntPtr src, uint nTlasNodes);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_trace_chunk_costs(IntPtr ctx, int bounce, uint* costs,
            uint max, out uint n);
        [DllImport(Lib)] public static extern TTStatus tt_async_overflows(IntPtr ctx, out ulong count);
        // per-call timing markers on (default) / off for asynchronous calls
        [DllImport(Lib)] public static extern TTStatus tt_ctx_set_timing(IntPtr ctx, int enabled);
        [DllImport(Lib)] public static extern TTStatus tt_ctx_set_frame_pixels(IntPtr ctx, uint framePixels);
        [DllImport(Lib)] public static extern IntPtr tt_ctx_stream(IntPtr ctx);
        // _AlphaAtlas texels (R8, row-major width x height), read back once per scene change.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_upload_alpha_atlas(IntPtr ctx, byte* texels,
            uint width, uint height);
        // _TextureAtlas decoded to RGBA half (4 x ushort per texel), for the stained-glass shadow tint.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_upload_texture_atlas(IntPtr ctx, ushort* rgbaHalf,
            uint width, uint height);
        // RefitTLAS: MeshAABBs as {BBMax.xyz, BBMin.xyz} per mesh; flags: TT_TRACE_DEVICE_PTRS / ASYNC.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_tlas_refit(IntPtr ctx, uint nTlasNodes, float* meshAabbs,
            uint nMesh, uint flags);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_read_nodes(IntPtr ctx, uint first, uint count, void* nodes);
        // ParentObject.RefitMesh: vertex buffer (floats), sharedMesh.triangles, CWBVHIndicesBufferInverted.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_blas_refit(IntPtr ctx, ref TTBlasRefitParams p, float* vertices,
            int* indices, int* leafOfTriangle);
        [DllImport(Lib)] public static extern TTStatus tt_sync(IntPtr ctx);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_read_tris(IntPtr ctx, uint first, uint count, void* tris);
        [DllImport(Lib)] public static extern TTStatus tt_scene_bytes(IntPtr ctx, out ulong bytes);
        // the structural check tt_scene_upload runs, without a GPU; `why` receives the first violation
        [DllImport(Lib)] public static extern unsafe TTStatus tt_scene_validate(void* nodes, uint nNodes, void* tris,
            uint nTris, int* tlasIndices, uint nTlas, void* meshData, uint nMesh, void* materials, uint nMat,
            byte* why, uint whyLen);
        // the producers either side of the trace (SURVEY.md §8 f2): Generate, and the diffuse next-bounce enqueue
        // with stable compaction into the other half of GlobalRays (host count, or device-resident counts)
        [DllImport(Lib)] public static extern TTStatus tt_generate_primary(IntPtr ctx, ref TTCamera cam, IntPtr globalRays);
        [DllImport(Lib)] public static extern TTStatus tt_enqueue_diffuse_bounce(IntPtr ctx, ref TTTraceParams p,
            IntPtr globalRays, int framesAccumulated, int maxBounce, out uint nNext);
        [DllImport(Lib)] public static extern TTStatus tt_enqueue_diffuse_bounce_indirect(IntPtr ctx, ref TTTraceParams p,
            IntPtr nRaysDev, IntPtr globalRays, int framesAccumulated, int maxBounce, IntPtr nNextDev);
        // GetTriangleNormal per hit: float[6] (shading xyz, geometric xyz) per ray
        [DllImport(Lib)] public static extern TTStatus tt_resolve_normals(IntPtr ctx, ref TTTraceParams p, IntPtr globalRays,
            IntPtr normals6);
        [DllImport(Lib)] public static extern TTStatus tt_timing_reset(IntPtr ctx);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_timing_read(IntPtr ctx, float* ms, uint max, out uint n);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_trace_diagnostics(IntPtr ctx, ulong* out8);
        [DllImport(Lib)] public static extern TTStatus tt_selftest_rcp(IntPtr ctx, out ulong mismatches);
        // multi-GPU tile-sharded frames (one process driving n devices, or one rank per process)
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_create(int* devices, uint n, ref TTGroupConfig cfg,
            out IntPtr group);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_unique_id(byte* id128);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_create_rank(byte* id128, uint world, uint rank,
            int device, ref TTGroupConfig cfg, out IntPtr group);
        [DllImport(Lib)] public static extern TTStatus tt_group_destroy(IntPtr group);
        [DllImport(Lib)] public static extern IntPtr tt_group_last_error(IntPtr group);
        [DllImport(Lib)] public static extern uint tt_group_local_members(IntPtr group);
        [DllImport(Lib)] public static extern IntPtr tt_group_member_ctx(IntPtr group, uint member);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_scene_upload(IntPtr group,
            void* nodes, uint nNodes, void* tris, uint nTris, int* tlasIndices, uint nTlas,
            void* meshData, uint nMesh, void* materials, uint nMat);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_scene_upload_alpha_atlas(IntPtr group, byte* texels,
            uint width, uint height);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_scene_upload_texture_atlas(IntPtr group,
            ushort* rgbaHalf, uint width, uint height);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_scene_update_meshdata(IntPtr group, uint first,
            uint count, void* meshData);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_scene_update_nodes(IntPtr group, uint first,
            uint count, void* nodes);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_tlas_refit(IntPtr group, uint nTlasNodes,
            float* meshAabbs, uint nMesh, uint flags);
        [DllImport(Lib)] public static extern TTStatus tt_group_trace_frame(IntPtr group, ref TTCamera cam, IntPtr hitsOut,
            IntPtr infoOut, uint flags);
        [DllImport(Lib)] public static extern TTStatus tt_group_sync(IntPtr group);
        [DllImport(Lib)] public static extern TTStatus tt_group_frame_rays(IntPtr group, uint member, out uint nPrimary,
            out uint nBounce, out IntPtr raysDev);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_group_tile_pixels(uint width, uint height, uint tile,
            uint world, uint rank, uint* pixels, uint max, out uint n);
        // BVH2Builder's three Array.Sort centroid presorts (introsort replayed, same tie order); returns
        // TTStatus.Unsupported for n <= 16 or non-finite centroids: then Array.Sort on the C# side.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_bvh2_presort_device(IntPtr ctx, float* aabbs, uint n,
            int* presorted);
        // ParentObject.BuildTotal's BVH2Builder + BVH8Builder + Aggregate on the GPU, after the presort
        // (byte-identical to the C# build): triangle AABBs {max, min}, 3 x n presorted indices, nodes out.
        [DllImport(Lib)] public static extern unsafe TTStatus tt_blas_build_device(IntPtr ctx, float* aabbs, uint n,
            int* presorted, void* nodes, uint maxNodes, out uint nNodes, int* cwbvhIndices, out uint bvh2Depth);
        [DllImport(Lib)] public static extern unsafe TTStatus tt_bvh2_build_device(IntPtr ctx, float* aabbs, uint n,
            int* presorted, int* finalIndices, float* nodeAabbs, int* nodeLeft, uint* nodeCount, out uint maxDepth);
    }

    /// A stream made by tt_stream_create, destroyed (tt_stream_destroy: synchronise + destroy) when released.
    public sealed class TTStreamHandle : SafeHandle
    {
        public TTStreamHandle() : base(IntPtr.Zero, true) { }
        public override bool IsInvalid => handle == IntPtr.Zero;
        protected override bool ReleaseHandle() => Native.tt_stream_destroy(handle) == TTStatus.Ok;
    }

    /// Replaces `cmd.DispatchCompute(IntersectionShader, TraceKernel, CurBounceInfoBuffer, 0)`
    /// (RayTracingMaster.cs:964-970) and the buffer binding of AssetManager.SetMeshTraceBuffers
    /// (AssetManager.cs:75-88) with calls into the HIP engine.
    public sealed class TrueTraceHipTracer : IDisposable
    {
        IntPtr m_ctx;
        TTStreamHandle m_stream;  // a tt_stream_create stream this tracer issues on, kept alive while it does
        bool m_streamRef;

        /// `hipStream`: the hipStream_t to issue on (IntPtr.Zero: a library-owned stream).
        public TrueTraceHipTracer(int device, ulong maxRays, IntPtr hipStream = default)
        {
            var cfg = new TTConfig { device = device, flags = 0, maxRays = maxRays, stream = hipStream };
            Check(Native.tt_ctx_create(ref cfg, out m_ctx));
        }

        /// Issue on a stream made by StreamCreate. The tracer holds a reference on the handle until it is
        /// disposed, so a dropped or finalized handle never destroys the stream under a live tracer.
        public TrueTraceHipTracer(int device, ulong maxRays, TTStreamHandle stream)
        {
            bool added = false;
            stream.DangerousAddRef(ref added);
            var cfg = new TTConfig { device = device, flags = 0, maxRays = maxRays, stream = stream.DangerousGetHandle() };
            var st = Native.tt_ctx_create(ref cfg, out m_ctx);
            if (st != TTStatus.Ok)
            {
                if (added) stream.DangerousRelease();
                throw new InvalidOperationException($"tt_ctx_create: {st}");
            }
            m_stream = stream;
            m_streamRef = added;
        }

        /// Raw context handle (e.g. for Native calls this wrapper does not cover).
        public IntPtr Handle => m_ctx;

        /// Generate (RayGenKernels.compute:40-57) into GlobalRays[pixel] on the device: the producer before the
        /// primary trace. `async` returns without waiting.
        public void GeneratePrimary(ref TTCamera cam, IntPtr globalRays, bool async = false)
        {
            cam.flags = TTTraceFlags.DevicePtrs | (async ? TTTraceFlags.Async : 0);
            Check(Native.tt_generate_primary(m_ctx, ref cam, globalRays));
        }

        /// The diffuse next-bounce enqueue after a trace of bounce `curBounce` (kernel_shade's next-ray
        /// production, RayTracingShader.compute:498-506): survivors compacted into the other ping-pong half;
        /// returns their count (synchronises).
        public uint EnqueueDiffuseBounce(IntPtr globalRays, uint nRays, int curBounce, float farPlane, int width, int height,
                                         int framesAccumulated, int maxBounce)
        {
            var p = new TTTraceParams { nRays = nRays, bounce = curBounce, farPlane = farPlane, screenWidth = (uint)width,
                                        screenHeight = (uint)height, flags = TTTraceFlags.DevicePtrs };
            Check(Native.tt_enqueue_diffuse_bounce(m_ctx, ref p, globalRays, framesAccumulated, maxBounce, out uint n));
            return n;
        }

        /// The same enqueue with device-resident counts (BufferSizes on the GPU): reads the traced count at
        /// `nRaysDevice` (IntPtr.Zero: `capacity`), writes the survivor count to `nNextDevice`; no host wait, so
        /// Generate -> TraceDevice -> EnqueueDiffuseBounceIndirect -> TraceDeviceIndirect is one device chain.
        public void EnqueueDiffuseBounceIndirect(IntPtr globalRays, IntPtr nRaysDevice, uint capacity, int curBounce,
                                                 float farPlane, int width, int height, int framesAccumulated,
                                                 int maxBounce, IntPtr nNextDevice)
        {
            var p = new TTTraceParams { nRays = capacity, bounce = curBounce, farPlane = farPlane, screenWidth = (uint)width,
                                        screenHeight = (uint)height, flags = TTTraceFlags.DevicePtrs };
            Check(Native.tt_enqueue_diffuse_bounce_indirect(m_ctx, ref p, nRaysDevice, globalRays, framesAccumulated,
                                                            maxBounce, nNextDevice));
        }

        /// GetTriangleNormal for every hit of a traced batch (float[6] per ray in HIP memory at `normals6`).
        public void ResolveNormals(IntPtr globalRays, uint nRays, int curBounce, float farPlane, int width, int height,
                                   IntPtr normals6)
        {
            var p = new TTTraceParams { nRays = nRays, bounce = curBounce, farPlane = farPlane, screenWidth = (uint)width,
                                        screenHeight = (uint)height, flags = TTTraceFlags.DevicePtrs };
            Check(Native.tt_resolve_normals(m_ctx, ref p, globalRays, normals6));
        }

        /// Per-call GPU times (HIP events) since the last TimingReset, in issue order.
        public void TimingReset() { Check(Native.tt_timing_reset(m_ctx)); }
        public unsafe float[] TimingRead()
        {
            var a = new float[256];
            uint n;
            fixed (float* p = a) Check(Native.tt_timing_read(m_ctx, p, 256, out n));
            Array.Resize(ref a, (int)n);
            return a;
        }

        /// tt_scene_validate: null when the buffers pass the upload's structural check, else the first violation.
        public static unsafe string Validate<TNode, TTri, TMesh, TMat>(TNode[] nodes, TTri[] tris, int[] tlasIndices,
                                                                       TMesh[] meshData, TMat[] materials)
            where TNode : unmanaged where TTri : unmanaged where TMesh : unmanaged where TMat : unmanaged
        {
            var why = new byte[512];
            TTStatus st;
            fixed (TNode* n = nodes) fixed (TTri* t = tris) fixed (int* i = tlasIndices)
            fixed (TMesh* m = meshData) fixed (TMat* mt = materials) fixed (byte* w = why)
                st = Native.tt_scene_validate(n, (uint)nodes.Length, t, (uint)tris.Length, i, (uint)tlasIndices.Length,
                                              m, (uint)meshData.Length, mt, (uint)materials.Length, w, (uint)why.Length);
            if (st == TTStatus.Ok) return null;
            int len = Array.IndexOf(why, (byte)0);
            return $"{st}: {System.Text.Encoding.ASCII.GetString(why, 0, len < 0 ? why.Length : len)}";
        }

        /// tt_shutdown: destroys every library stream still alive. Call from OnApplicationQuit (or
        /// AppDomain.DomainUnload) when dispatches come from a thread other than the main one, after the last one.
        public static void Shutdown() { Native.tt_shutdown(); }

        /// The hipStream_t the engine issues on (for ordering the caller's own HIP work around it).
        public IntPtr Stream => Native.tt_ctx_stream(m_ctx);

        /// AssetManager.SetMeshTraceBuffers: the same arrays the AssetManager uploads with
        /// ComputeBuffer.SetData (AssetManager.cs:1760, :1762; ParentObject.cs:270-271).
        public unsafe void SetMeshTraceBuffers<TNode, TTri, TMesh, TMat>(TNode[] nodes, TTri[] tris, int[] tlasIndices,
                                                                        TMesh[] meshData, TMat[] materials)
            where TNode : unmanaged where TTri : unmanaged where TMesh : unmanaged where TMat : unmanaged
        {
            fixed (TNode* n = nodes) fixed (TTri* t = tris) fixed (int* i = tlasIndices)
            fixed (TMesh* m = meshData) fixed (TMat* mt = materials)
                Check(Native.tt_scene_upload(m_ctx, n, (uint)nodes.Length, t, (uint)tris.Length, i, (uint)tlasIndices.Length,
                                             m, (uint)meshData.Length, mt, (uint)materials.Length));
        }

        /// One kernel_trace dispatch for bounce `curBounce`.
        public unsafe TTStats Trace<TRay, TCol>(TRay[] globalRays, uint nRays, int curBounce, float farPlane,
                                                int width, int height, uint[] primaryInfo = null, TCol[] globalColors = null,
                                                bool useReSTIRGI = false, bool useASVGF = false)
            where TRay : unmanaged where TCol : unmanaged
        {
            var p = new TTTraceParams
            {
                nRays = nRays, bounce = curBounce, farPlane = farPlane, screenWidth = (uint)width, screenHeight = (uint)height,
                flags = (useReSTIRGI ? TTTraceFlags.UseReSTIRGI : 0) | (useASVGF ? TTTraceFlags.UseASVGF : 0)
            };
            TTStats s;
            fixed (TRay* r = globalRays) fixed (uint* info = primaryInfo) fixed (TCol* col = globalColors)
                Check(Native.tt_trace_closest(m_ctx, ref p, r, info, col, out s));
            return s;
        }

        /// One kernel_trace dispatch on buffers that already live in HIP device memory (a HIP-resident
        /// wavefront): no PCIe round trip of the 2*W*H RayData buffer. `async` returns without waiting
        /// (stack overflows of async launches: AsyncOverflows()).
        public TTStats TraceDevice(IntPtr globalRays, uint nRays, int curBounce, float farPlane, int width, int height,
                                   IntPtr primaryInfo = default, IntPtr globalColors = default,
                                   TTTraceFlags extra = TTTraceFlags.None, bool async = false)
        {
            var p = new TTTraceParams
            {
                nRays = nRays, bounce = curBounce, farPlane = farPlane, screenWidth = (uint)width, screenHeight = (uint)height,
                flags = extra | TTTraceFlags.DevicePtrs | (async ? TTTraceFlags.Async : 0)
            };
            Check(Native.tt_trace_closest_dev(m_ctx, ref p, globalRays, primaryInfo, globalColors, out TTStats s));
            return s;
        }

        /// Trace `lender`'s scene on this context's stream without a copy (tt_ctx_share_scene): e.g. the second
        /// half of a frame traced concurrently on its own context. Update the scene through the lender;
        /// dispose this context before the lender.
        public void ShareScene(TrueTraceHipTracer lender) { Check(Native.tt_ctx_share_scene(m_ctx, lender.m_ctx)); }

        /// A frame slot over `lender`'s scene (tt_ctx_share_blas): the lender's BLASes and triangles without a copy,
        /// under a TLAS, TLASBVH8Indices and _MeshData of this context's own (copied now). This frame's
        /// RefitTLAS / SetMeshData on THIS tracer (AssetManager.cs:1821-1825) then neither wait for nor touch the
        /// other frames in flight. `tlasNodeCount`: the TLAS region at the front of the node array.
        public void ShareBlas(TrueTraceHipTracer lender, uint tlasNodeCount)
        {
            Check(Native.tt_ctx_share_blas(m_ctx, lender.m_ctx, tlasNodeCount));
        }

        /// Per-call GPU timing (tt_ctx_set_timing): off, asynchronous calls put no event markers around their
        /// kernels -- the setting for every frame-slot context but the one a host measures, if any.
        public void SetTiming(bool enabled) { Check(Native.tt_ctx_set_timing(m_ctx, enabled ? 1 : 0)); }
        /// Batched frames on a B-tall screen (tt_ctx_set_frame_pixels): frame j's bounce random numbers are
        /// those of its own pixel at frames + j; 0 = PixelIndex as-is.
        public void SetFramePixels(uint framePixels) { Check(Native.tt_ctx_set_frame_pixels(m_ctx, framePixels)); }

        /// The per-64-ray-chunk costs the last AdaptiveOrder trace of `bounce` recorded (tt_trace_chunk_costs): one
        /// value per 8x8 pixel tile for a full-frame launch -- the input of a multi-GPU host's tile balancing.
        public unsafe uint[] ChunkCosts(int bounce, uint maxChunks)
        {
            var a = new uint[maxChunks];
            uint n;
            fixed (uint* p = a) Check(Native.tt_trace_chunk_costs(m_ctx, bounce, p, maxChunks, out n));
            Array.Resize(ref a, (int)n);
            return a;
        }

        /// A hipStream_t on a hardware queue of its own (tt_stream_create) for a concurrently traced half of
        /// the frame: pass the handle to that half's tracer (the TTStreamHandle constructor, which keeps it alive
        /// until the tracer is disposed). The handle is a SafeHandle: a finalizer or a domain reload that skips
        /// Dispose still destroys the stream (and the library destroys any stream left at process exit).
        public static TTStreamHandle StreamCreate(int device)
        {
            var st = Native.tt_stream_create(device, out TTStreamHandle s);
            if (st != TTStatus.Ok)
            {
                s?.SetHandleAsInvalid();
                throw new InvalidOperationException($"tt_stream_create: {st}");
            }
            return s;
        }
        public static void StreamDestroy(TTStreamHandle stream) { stream?.Dispose(); }

        /// TraceDevice that also writes ray i's 16-byte hit record to hitsOut[i] (HIP device memory, 16-byte
        /// aligned, nRays records): the buffer a multi-GPU host gathers (tt_trace_closest_hits).
        public void TraceDeviceHits(IntPtr globalRays, uint nRays, int curBounce, float farPlane, int width, int height,
                                    IntPtr hitsOut, IntPtr primaryInfo = default, IntPtr globalColors = default,
                                    TTTraceFlags extra = TTTraceFlags.None, bool async = false)
        {
            var p = new TTTraceParams
            {
                nRays = nRays, bounce = curBounce, farPlane = farPlane, screenWidth = (uint)width, screenHeight = (uint)height,
                flags = extra | TTTraceFlags.DevicePtrs | (async ? TTTraceFlags.Async : 0)
            };
            Check(Native.tt_trace_closest_hits(m_ctx, ref p, globalRays, primaryInfo, globalColors, hitsOut));
        }

        /// kernel_trace as DispatchIndirect: the ray count is the uint at `nRaysDevice` (HIP device memory,
        /// written by an earlier operation on the context stream, e.g. the shading pass's BufferSizes),
        /// clamped to `capacity`; the call never waits for the GPU.
        public void TraceDeviceIndirect(IntPtr globalRays, IntPtr nRaysDevice, uint capacity, int curBounce, float farPlane,
                                        int width, int height, IntPtr primaryInfo = default, IntPtr globalColors = default,
                                        TTTraceFlags extra = TTTraceFlags.None)
        {
            var p = new TTTraceParams
            {
                nRays = capacity, bounce = curBounce, farPlane = farPlane, screenWidth = (uint)width, screenHeight = (uint)height,
                flags = extra | TTTraceFlags.DevicePtrs
            };
            Check(Native.tt_trace_closest_indirect(m_ctx, ref p, nRaysDevice, globalRays, primaryInfo, globalColors));
        }

        /// tt_trace_shadow (the original signature and contract): visibility, t write-back,
        /// Direct += at bounce 0 and NEEPosA only; the caller does the other :457-485 accumulations.
        public unsafe TTStats TraceShadow<TShadow, TCol>(TShadow[] shadowRays, uint nRays, int curBounce, int width,
                                                         int height, float[] visibility = null,
                                                         TCol[] globalColors = null, float[] neePos = null,
                                                         TTTraceFlags flags = 0)
            where TShadow : unmanaged where TCol : unmanaged
        {
            var p = new TTShadowParams { nRays = nRays, bounce = curBounce, screenWidth = (uint)width,
                                         screenHeight = (uint)height, flags = flags };
            TTStats s;
            fixed (TShadow* r = shadowRays) fixed (float* vis = visibility) fixed (TCol* col = globalColors)
            fixed (float* nee = neePos)
                Check(Native.tt_trace_shadow(m_ctx, ref p, r, vis, col, nee, out s));
            return s;
        }

        /// One kernel_shadow dispatch (IntersectionKernels.compute:264-505) for bounce `curBounce`
        /// with the full :457-485 output contract (tt_trace_shadow_ex); `cacheBuffer`
        /// (PropogatedCacheData per pixel) and `flags` (RadianceCache, VisibilityCheck, UseReSTIRGI)
        /// select the accumulations of the reference's define set.
        public unsafe TTStats TraceShadowEx<TShadow, TCol, TCache>(TShadow[] shadowRays, uint nRays, int curBounce, int width,
                                                                   int height, float[] visibility = null,
                                                                   TCol[] globalColors = null, float[] neePos = null,
                                                                   TCache[] cacheBuffer = null,
                                                                   TTTraceFlags flags = TTTraceFlags.RadianceCache)
            where TShadow : unmanaged where TCol : unmanaged where TCache : unmanaged
        {
            var p = new TTShadowParams { nRays = nRays, bounce = curBounce, screenWidth = (uint)width,
                                         screenHeight = (uint)height, flags = flags };
            TTStats s;
            fixed (TShadow* r = shadowRays) fixed (float* vis = visibility) fixed (TCol* col = globalColors)
            fixed (float* nee = neePos) fixed (TCache* cache = cacheBuffer)
                Check(Native.tt_trace_shadow_ex(m_ctx, ref p, r, vis, col, nee, cache, out s));
            return s;
        }

        /// TraceShadow on HIP device buffers (no host round trip).
        public TTStats TraceShadowDevice(IntPtr shadowRays, uint nRays, int curBounce, int width, int height,
                                         IntPtr visibility = default, IntPtr globalColors = default, IntPtr neePos = default,
                                         IntPtr cacheBuffer = default, TTTraceFlags flags = TTTraceFlags.RadianceCache,
                                         bool async = false)
        {
            var p = new TTShadowParams { nRays = nRays, bounce = curBounce, screenWidth = (uint)width,
                                         screenHeight = (uint)height,
                                         flags = flags | TTTraceFlags.DevicePtrs | (async ? TTTraceFlags.Async : 0) };
            Check(Native.tt_trace_shadow_dev(m_ctx, ref p, shadowRays, visibility, globalColors, neePos, cacheBuffer,
                                             out TTStats s));
            return s;
        }

        /// Stack overflows of every launch since the last call (TT_TRACE_ASYNC chains included).
        public ulong AsyncOverflows()
        {
            var st = Native.tt_async_overflows(m_ctx, out ulong n);
            if (st != TTStatus.StackOverflow) Check(st);
            return n;
        }

        /// The _AlphaAtlas binding of SetMeshTraceBuffers (AssetManager.cs:75-88): R8 texels, once
        /// per scene change, before tracing scenes with Cutout materials.
        public unsafe void SetAlphaAtlas(byte[] texels, int width, int height)
        {
            fixed (byte* t = texels)
                Check(Native.tt_scene_upload_alpha_atlas(m_ctx, t, (uint)width, (uint)height));
        }

        /// The _TextureAtlas binding of SetMeshTraceBuffers (AssetManager.cs:82): the BC6H albedo atlas
        /// decoded to RGBA half texels (e.g. Graphics.Blit into an RGBAHalf RenderTexture, then
        /// AsyncGPUReadback), once per scene change, before tracing shadows through glass materials.
        public unsafe void SetTextureAtlas(ushort[] rgbaHalf, int width, int height)
        {
            fixed (ushort* t = rgbaHalf)
                Check(Native.tt_scene_upload_texture_atlas(m_ctx, t, (uint)width, (uint)height));
        }

        /// AssetManager.RefitTLAS(Boxes, cmd) (AssetManager.cs:1473-1548): re-quantizes the TLAS
        /// nodes in HBM from this frame's MeshAABBs (6 floats per mesh: BBMax, BBMin).
        public unsafe void RefitTLAS(float[] meshAabbs, int nTlasNodes)
        {
            fixed (float* b = meshAabbs)
                Check(Native.tt_tlas_refit(m_ctx, (uint)nTlasNodes, b, (uint)(meshAabbs.Length / 6), 0));
        }

        /// ParentObject.RefitMesh (ParentObject.cs:750-917) for a skinned / deformable mesh: pass the
        /// vertex buffer read back from SkinnedMeshRenderer.GetVertexBuffer (floats), the mesh's
        /// triangles, CWBVHIndicesBufferInverted and the "Transform" matrix; RefitTLAS follows.
        public unsafe void RefitMesh(int meshIndex, float[] vertices, int vertexStride, int[] triangles,
                                     int[] leafOfTriangle, Matrix4x4Floats transform)
        {
            var p = new TTBlasRefitParams { meshIndex = (uint)meshIndex, nTris = (uint)(triangles.Length / 3),
                                            nVertices = (uint)(vertices.Length / vertexStride),
                                            vertexStride = (uint)vertexStride, flags = 0 };
            for (int i = 0; i < 16; i++) p.transform[i] = transform.m[i];
            fixed (float* v = vertices) fixed (int* t = triangles) fixed (int* l = leafOfTriangle)
                Check(Native.tt_blas_refit(m_ctx, ref p, v, t, l));
        }

        void Check(TTStatus st)
        {
            if (st != TTStatus.Ok)
                throw new InvalidOperationException($"truetrace_hip: {st}: {Marshal.PtrToStringAnsi(Native.tt_last_error(m_ctx))}");
        }

        public void Dispose()
        {
            if (m_ctx != IntPtr.Zero) { Native.tt_ctx_destroy(m_ctx); m_ctx = IntPtr.Zero; }
            if (m_streamRef) { m_stream.DangerousRelease(); m_streamRef = false; }
            m_stream = null;
        }
    }

    /// C5's multi-GPU mode behind the C ABI (tt_group_*): the scene replicated per device, a frame's 64x64 tiles
    /// dealt round-robin, each device generating and tracing its tiles (and their bounce 1), and the primary hit
    /// records gathered to device 0 in screen order with one RCCL gather. Replaces, for a whole frame, the
    /// Generate + per-bounce kernel_trace dispatches of RayTracingMaster.RenderImage (RayTracingMaster.cs:954-1007).
    public sealed class TrueTraceHipGroup : IDisposable
    {
        IntPtr m_g;

        /// One process driving `devices` (member 0 receives the gather).
        public unsafe TrueTraceHipGroup(int[] devices, TTGroupConfig cfg)
        {
            fixed (int* d = devices) Check(Native.tt_group_create(d, (uint)devices.Length, ref cfg, out m_g));
        }

        /// One rank per process: every process calls this with rank 0's UniqueId() (the host distributes it).
        public unsafe TrueTraceHipGroup(byte[] uniqueId, uint world, uint rank, int device, TTGroupConfig cfg)
        {
            fixed (byte* id = uniqueId) Check(Native.tt_group_create_rank(id, world, rank, device, ref cfg, out m_g));
        }

        public static unsafe byte[] UniqueId()
        {
            var id = new byte[128];
            fixed (byte* p = id)
                if (Native.tt_group_unique_id(p) != TTStatus.Ok) throw new InvalidOperationException("tt_group_unique_id");
            return id;
        }

        /// AssetManager.SetMeshTraceBuffers on every device of the group (the scene replicated).
        public unsafe void SetMeshTraceBuffers<TNode, TTri, TMesh, TMat>(TNode[] nodes, TTri[] tris, int[] tlasIndices,
                                                                        TMesh[] meshData, TMat[] materials)
            where TNode : unmanaged where TTri : unmanaged where TMesh : unmanaged where TMat : unmanaged
        {
            fixed (TNode* n = nodes) fixed (TTri* t = tris) fixed (int* i = tlasIndices)
            fixed (TMesh* m = meshData) fixed (TMat* mt = materials)
                Check(Native.tt_group_scene_upload(m_g, n, (uint)nodes.Length, t, (uint)tris.Length, i, (uint)tlasIndices.Length,
                                                   m, (uint)meshData.Length, mt, (uint)materials.Length));
        }

        /// Per-frame MeshDataBuffer.SetData + RefitTLAS (AssetManager.cs:1767-1826) on every device, between frames.
        public unsafe void SetMeshData<TMesh>(TMesh[] meshData) where TMesh : unmanaged
        {
            fixed (TMesh* m = meshData) Check(Native.tt_group_scene_update_meshdata(m_g, 0, (uint)meshData.Length, m));
        }
        public unsafe void RefitTLAS(float[] meshAabbs, int nTlasNodes)
        {
            fixed (float* b = meshAabbs)
                Check(Native.tt_group_tlas_refit(m_g, (uint)nTlasNodes, b, (uint)(meshAabbs.Length / 6), 0));
        }

        /// The _AlphaAtlas / decoded _TextureAtlas on every device (after SetMeshTraceBuffers).
        public unsafe void SetAlphaAtlas(byte[] texels, int width, int height)
        {
            fixed (byte* t = texels) Check(Native.tt_group_scene_upload_alpha_atlas(m_g, t, (uint)width, (uint)height));
        }
        public unsafe void SetTextureAtlas(ushort[] rgbaHalf, int width, int height)
        {
            fixed (ushort* t = rgbaHalf) Check(Native.tt_group_scene_upload_texture_atlas(m_g, t, (uint)width, (uint)height));
        }

        /// One frame: Generate + primary trace per device for its tiles, the gather of the primary hit records to
        /// `hitsOut` (device 0, width*height uint4 in screen order), bounce 1 per device with TTGroupFlags.Bounce;
        /// with TTGroupFlags.Info the bounce-0 _PrimaryTriangleInfo texels go to `infoOut` the same way.
        public void TraceFrame(ref TTCamera cam, IntPtr hitsOut, IntPtr infoOut = default, bool async = false)
        {
            Check(Native.tt_group_trace_frame(m_g, ref cam, hitsOut, infoOut, async ? (uint)TTTraceFlags.Async : 0u));
        }

        public void Sync() { Check(Native.tt_group_sync(m_g)); }

        /// Member m's scene context: per-frame scene updates (RefitTLAS, SetMeshData) go through it.
        public IntPtr MemberContext(uint m) => Native.tt_group_member_ctx(m_g, m);
        public uint LocalMembers => Native.tt_group_local_members(m_g);

        /// The latest frame of member m: primary and bounce-1 counts and its RayData buffer in HIP memory.
        public (uint primary, uint bounce, IntPtr rays) FrameRays(uint m)
        {
            Check(Native.tt_group_frame_rays(m_g, m, out uint a, out uint b, out IntPtr r));
            return (a, b, r);
        }

        void Check(TTStatus st)
        {
            if (st != TTStatus.Ok)
                throw new InvalidOperationException(
                    $"truetrace_hip group: {st}: {(m_g == IntPtr.Zero ? "" : Marshal.PtrToStringAnsi(Native.tt_group_last_error(m_g)))}");
        }

        public void Dispose()
        {
            if (m_g != IntPtr.Zero) { Native.tt_group_destroy(m_g); m_g = IntPtr.Zero; }
        }
    }
}
