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

    /// Column-major 4x4 (the memory order of UnityEngine.Matrix4x4: m00, m10, m20, m30, m01, ...).
    public struct Matrix4x4Floats { public float[] m; }

    public static class Native
    {
        const string Lib = "truetrace_hip";
        [DllImport(Lib)] public static extern TTStatus tt_ctx_create(ref TTConfig cfg, out IntPtr ctx);
        [DllImport(Lib)] public static extern TTStatus tt_ctx_destroy(IntPtr ctx);
        [DllImport(Lib)] public static extern IntPtr tt_last_error(IntPtr ctx);
        [DllImport(Lib)] public static extern int tt_device_count();
        [DllImport(Lib)] public static extern TTStatus tt_stream_create(int device, out TTStreamHandle stream);
        [DllImport(Lib)] public static extern TTStatus tt_stream_destroy(IntPtr stream);
        [DllImport(Lib)] public static extern uint tt_stream_live_count();
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

        /// `hipStream`: the hipStream_t to issue on (IntPtr.Zero: a library-owned stream).
        public TrueTraceHipTracer(int device, ulong maxRays, IntPtr hipStream = default)
        {
            var cfg = new TTConfig { device = device, flags = 0, maxRays = maxRays, stream = hipStream };
            Check(Native.tt_ctx_create(ref cfg, out m_ctx));
        }

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
        /// the frame: pass handle.DangerousGetHandle() as the hipStream of that half's tracer and dispose the
        /// handle after the tracer. The handle is a SafeHandle: a finalizer or a domain reload that skips
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
        }
    }
}
