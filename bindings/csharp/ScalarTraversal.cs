// ScalarTraversal.cs — the north star's "scalar C#" CPU baseline (SURVEY.md §8(d)): a one-ray-at-a-
// time C# restatement of the closest-hit path (kernel_trace / IntersectBVH,
// IntersectionKernels.compute:60-254; IntersectTriangle :14-57; cwbvh_node_intersect
// CommonData.cginc:641-707) over the exact buffers AssetManager.SetMeshTraceBuffers binds
// (80 B nodes, 88 B CudaTriangle, TLASBVH8Indices, 88 B MyMeshDataCompacted, 252 B materials),
// with the numerics of SURVEY.md appendix A (IEEE 1/x, explicit FMA, minNum/maxNum, no contraction)
// — the same semantics as oracle/tt_oracle.c and the gfx950 kernel.
//
// It is a baseline, not a product path: no .NET runtime exists in the build image or on the GPU
// box, so bench.py reports "C# scalar baseline not run". With .NET 6+:
//     python tools/dump_scene_raw.py /tmp/c2      # C2 scene + 1080p primary rays + oracle hits
//     dotnet run -c Release -- /tmp/c2 [threads]  # (a console project containing this file)
// prints Mrays/s and checks every hit record against the oracle's.
// Scope: opaque + Invisible-at-bounce-0 materials (Cutout needs the alpha atlas: reported unsupported).

using System;
using System.Diagnostics;
using System.IO;
using System.Numerics;
using System.Runtime.InteropServices;
using System.Threading.Tasks;

namespace TrueTraceHip
{
    public sealed class TraceBuffers
    {
        public uint[] Nodes;      // 20 words per node
        public uint[] Tris;       // 22 words per triangle
        public int[] Tlas;        // TLASBVH8Indices
        public uint[] MeshData;   // 22 words per mesh
        public uint[] Materials;  // 63 words per material
        public int NMat => Materials.Length / 63;
    }

    public static class ScalarTraversal
    {
        public const int StackSize = 16;    // uint2 stack[16], IntersectionKernels.compute:65
        public const int MaxReps = 1000;    // while (Reps < 1000)
        const int MatTagWord = 23;          // Tag @92
        const int MatTypeWord = 25;         // MatType @100
        const int CutoutIndex = 2;          // GlobalDefines.cginc:24
        const int InvisibleBit = 7;         // GlobalDefines.cginc:46

        struct Ray { public float ox, oy, oz, dx, dy, dz, ix, iy, iz; }

        static float F(uint u) => BitConverter.Int32BitsToSingle((int)u);
        static uint U(float f) => (uint)BitConverter.SingleToInt32Bits(f);
        static float Fma(float a, float b, float c) => MathF.FusedMultiplyAdd(a, b, c);
        // IEEE minNum / maxNum: a NaN operand yields the other operand (DXIL min/max)
        static float MaxNum(float a, float b) => float.IsNaN(a) ? b : float.IsNaN(b) ? a : (a > b ? a : b);
        static float MinNum(float a, float b) => float.IsNaN(a) ? b : float.IsNaN(b) ? a : (a < b ? a : b);
        static uint FirstBitHigh(uint x) => 31u - (uint)BitOperations.LeadingZeroCount(x);

        static uint OctantInv4(float dx, float dy, float dz) =>     // CommonData.cginc:635-640
            (dx < 0.0f ? 0u : 0x04040404u) | (dy < 0.0f ? 0u : 0x02020202u) | (dz < 0.0f ? 0u : 0x01010101u);

        static void SetInverse(ref Ray r) { r.ix = 1.0f / r.dx; r.iy = 1.0f / r.dy; r.iz = 1.0f / r.dz; }

        // cwbvh_node_intersect — CommonData.cginc:641-707
        static uint NodeIntersect(uint[] N, int b, in Ray r, uint octInv4, float maxDistance)
        {
            uint w = N[b + 3];
            float ax = F((w & 0xffu) << 23) * r.ix, ay = F(((w >> 8) & 0xffu) << 23) * r.iy,
                  az = F(((w >> 16) & 0xffu) << 23) * r.iz;
            float ox = r.ix * (F(N[b]) - r.ox), oy = r.iy * (F(N[b + 1]) - r.oy), oz = r.iz * (F(N[b + 2]) - r.oz);
            uint hitMask = 0;
            for (int i = 0; i < 2; i++)
            {
                uint meta4 = N[b + 6 + i];
                uint isInner4 = (meta4 & (meta4 << 1)) & 0x10101010u;
                uint innerMask4 = (((isInner4 << 3) >> 7) & 0x01010101u) * 0xffu;
                uint bitIndex4 = (meta4 ^ (octInv4 & innerMask4)) & 0x1f1f1f1fu;
                uint childBits4 = (meta4 >> 5) & 0x07070707u;
                uint qlx = N[b + 8 + i], qhx = N[b + 10 + i], qly = N[b + 12 + i], qhy = N[b + 14 + i];
                uint qlz = N[b + 16 + i], qhz = N[b + 18 + i];
                uint xmin = r.dx < 0.0f ? qhx : qlx, xmax = r.dx < 0.0f ? qlx : qhx;
                uint ymin = r.dy < 0.0f ? qhy : qly, ymax = r.dy < 0.0f ? qly : qhy;
                uint zmin = r.dz < 0.0f ? qhz : qlz, zmax = r.dz < 0.0f ? qlz : qhz;
                for (int j = 0; j < 4; j++)
                {
                    int s = j * 8;
                    float t0x = Fma((float)((xmin >> s) & 0xffu), ax, ox);
                    float t0y = Fma((float)((ymin >> s) & 0xffu), ay, oy);
                    float t0z = Fma((float)((zmin >> s) & 0xffu), az, oz);
                    float t1x = Fma((float)((xmax >> s) & 0xffu), ax, ox);
                    float t1y = Fma((float)((ymax >> s) & 0xffu), ay, oy);
                    float t1z = Fma((float)((zmax >> s) & 0xffu), az, oz);
                    float tmin = MaxNum(MaxNum(t0x, t0y), MaxNum(t0z, 1e-8f));   // EPSILON, CommonData.cginc:3
                    float tmax = MinNum(MinNum(t1x, t1y), MinNum(t1z, maxDistance));
                    if (tmin < tmax)
                        hitMask |= ((childBits4 >> s) & 0xffu) << (int)((bitIndex4 >> s) & 0xffu);
                }
            }
            return hitMask;
        }

        static float Dot(float ax, float ay, float az, float bx, float by, float bz) => Fma(az, bz, Fma(ay, by, ax * bx));

        // IntersectTriangle — IntersectionKernels.compute:14-57. false = unsupported material reached.
        static bool IntersectTriangle(TraceBuffers S, int meshId, int triId, in Ray r, ref float bt, ref float bu,
                                      ref float bv, ref int bMesh, ref int bTri, int matOffset, int bounce)
        {
            uint[] T = S.Tris;
            int o = triId * 22;
            float p0x = F(T[o]), p0y = F(T[o + 1]), p0z = F(T[o + 2]);
            float e1x = F(T[o + 3]), e1y = F(T[o + 4]), e1z = F(T[o + 5]);
            float e2x = F(T[o + 6]), e2y = F(T[o + 7]), e2z = F(T[o + 8]);
            float hx = Fma(r.dy, e2z, -(r.dz * e2y)), hy = Fma(r.dz, e2x, -(r.dx * e2z)), hz = Fma(r.dx, e2y, -(r.dy * e2x));
            float a = Dot(e1x, e1y, e1z, hx, hy, hz);
            float f = 1.0f / a;
            float sx = r.ox - p0x, sy = r.oy - p0y, sz = r.oz - p0z;
            float u = f * Dot(sx, sy, sz, hx, hy, hz);
            if (u >= 0.0f && u <= 1.0f)
            {
                float qx = Fma(sy, e1z, -(sz * e1y)), qy = Fma(sz, e1x, -(sx * e1z)), qz = Fma(sx, e1y, -(sy * e1x));
                float v = f * Dot(r.dx, r.dy, r.dz, qx, qy, qz);
                if (v >= 0.0f && u + v <= 1.0f)
                {
                    float t = f * Dot(e2x, e2y, e2z, qx, qy, qz);
                    if (t > 0 && t < bt)
                    {
                        int mi = matOffset + (int)T[o + 21];
                        if (mi >= 0 && mi < S.NMat)  // out-of-range StructuredBuffer reads return zeros
                        {
                            int mo = mi * 63;
                            if ((int)S.Materials[mo + MatTypeWord] == CutoutIndex) return false;
                            if (bounce == 0 && (((int)S.Materials[mo + MatTagWord] >> InvisibleBit) & 1) == 1) return true;
                        }
                        bt = t; bu = u; bv = v; bMesh = meshId; bTri = triId;
                    }
                }
            }
            return true;
        }

        static void MeshRay(uint[] MD, int m, in Ray w, out Ray r)
        {
            int o = m * 22;  // W2L column-major: (row, col) at o + col*4 + row
            float M(int row, int col) => F(MD[o + col * 4 + row]);
            r = default;
            r.dx = Fma(M(0, 2), w.dz, Fma(M(0, 1), w.dy, M(0, 0) * w.dx));
            r.dy = Fma(M(1, 2), w.dz, Fma(M(1, 1), w.dy, M(1, 0) * w.dx));
            r.dz = Fma(M(2, 2), w.dz, Fma(M(2, 1), w.dy, M(2, 0) * w.dx));
            r.ox = Fma(M(0, 2), w.oz, Fma(M(0, 1), w.oy, M(0, 0) * w.ox)) + M(0, 3);
            r.oy = Fma(M(1, 2), w.oz, Fma(M(1, 1), w.oy, M(1, 0) * w.ox)) + M(1, 3);
            r.oz = Fma(M(2, 2), w.oz, Fma(M(2, 1), w.oy, M(2, 0) * w.ox)) + M(2, 3);
            SetInverse(ref r);
        }

        /// <summary>IntersectBVH for one ray (bounce-0 info only). rays: 12 words per RayData; hits
        /// written in place at words 8..11. Returns 0 done, 1 Reps exhausted (no write), 2 stack
        /// overflow, 3 unsupported material.</summary>
        public static int TraceRay(TraceBuffers S, uint[] rays, int rayIndex, int bounce, float farPlane,
                                   int width, int height, uint[] info)
        {
            int ro = rayIndex * 12;
            Ray ray = new Ray { ox = F(rays[ro]), oy = F(rays[ro + 1]), oz = F(rays[ro + 2]),
                                dx = F(rays[ro + 4]), dy = F(rays[ro + 5]), dz = F(rays[ro + 6]) };
            SetInverse(ref ray);
            Ray world = ray;
            float bt = farPlane, bu = 0, bv = 0;
            int bMesh = 0, bTri = -1;                                // CreateRayHit, CommonData.cginc:364-372
            Span<ulong> stack = stackalloc ulong[StackSize];         // (x | y << 32)
            int sp = 0, tlasSp = -1, nodeOffset = 0, triOffset = 0, matOffset = 0, meshId = -1;
            uint octInv4 = OctantInv4(ray.dx, ray.dy, ray.dz);
            uint gx = 0, gy = 0x80000000u, tx = 0, ty = 0;
            for (int reps = 0; reps < MaxReps;)
            {
                if ((gy & 0xff000000u) != 0)
                {   // :157-187
                    uint off = FirstBitHigh(gy);
                    uint slot = (off - 24) ^ (octInv4 & 0xffu);
                    uint rel = (uint)BitOperations.PopCount(gy & ~(0xffffffffu << (int)slot));
                    int child = (int)(gx + rel);
                    gy &= ~(1u << (int)off);
                    if ((gy & 0xff000000u) != 0)
                    {
                        if (sp == StackSize) return 2;
                        stack[sp++] = gx | ((ulong)gy << 32);
                    }
                    int nb = child * 20;
                    uint hit = NodeIntersect(S.Nodes, nb, ray, octInv4, bt);
                    gy = (hit & 0xff000000u) | ((S.Nodes[nb + 3] >> 24) & 0xffu);
                    ty = hit & 0x00ffffffu;
                    gx = S.Nodes[nb + 4] + (uint)nodeOffset;
                    tx = S.Nodes[nb + 5] + (uint)triOffset;
                    reps++;
                }
                else
                {   // :188-191
                    tx = gx; ty = gy; gx = 0; gy = 0;
                }
                if (ty != 0)
                {
                    if (tlasSp == -1)
                    {   // :194-219 TLAS leaf -> BLAS
                        uint mo = FirstBitHigh(ty);
                        ty &= ~(1u << (int)mo);
                        meshId = S.Tlas[tx + mo];
                        int m = meshId * 22;
                        nodeOffset = (int)S.MeshData[m + 17];
                        triOffset = (int)S.MeshData[m + 16];
                        if (ty != 0) { if (sp == StackSize) return 2; stack[sp++] = tx | ((ulong)ty << 32); }
                        if ((gy & 0xff000000u) != 0) { if (sp == StackSize) return 2; stack[sp++] = gx | ((ulong)gy << 32); }
                        tlasSp = sp;
                        matOffset = (int)S.MeshData[m + 18];
                        MeshRay(S.MeshData, meshId, world, out ray);
                        octInv4 = OctantInv4(ray.dx, ray.dy, ray.dz);
                        gx = S.MeshData[m + 19] & 0x7fffffffu;
                        gy = 0x80000000u;
                    }
                    else
                    {   // :220-226 leaf triangles, highest bit first
                        while (ty != 0)
                        {
                            uint ti = FirstBitHigh(ty);
                            ty &= ~(1u << (int)ti);
                            if (!IntersectTriangle(S, meshId, (int)(tx + ti), ray, ref bt, ref bu, ref bv, ref bMesh,
                                                   ref bTri, matOffset, bounce))
                                return 3;
                        }
                    }
                }
                if ((gy & 0xff000000u) == 0)
                {
                    if (sp == 0)
                    {   // :229-241
                        if (info != null && bounce == 0)
                        {
                            uint pix = rays[ro + 3];
                            uint px = pix % (uint)width, py = pix / (uint)width;
                            if (py < (uint)height)
                            {
                                int io = 4 * (int)(py * (uint)width + px);
                                info[io] = (uint)bMesh;
                                info[io + 1] = (uint)(bTri - (int)S.MeshData[bMesh * 22 + 16]);
                                info[io + 2] = U(bu);
                                info[io + 3] = U(bv);
                            }
                        }
                        rays[ro + 8] = (uint)bMesh;                     // set(), CommonData.cginc:430-434
                        rays[ro + 9] = (uint)bTri;
                        rays[ro + 10] = U(bt);
                        rays[ro + 11] = (uint)(bu * 65535.0f) | ((uint)(bv * 65535.0f) << 16);
                        return 0;
                    }
                    if (sp == tlasSp)
                    {   // :243-249 BLAS -> TLAS
                        nodeOffset = 0; triOffset = 0; tlasSp = -1;
                        ray = world;
                        octInv4 = OctantInv4(ray.dx, ray.dy, ray.dz);
                    }
                    ulong g = stack[--sp];
                    gx = (uint)g; gy = (uint)(g >> 32);
                }
            }
            return 1;
        }

        /// <summary>Traces rays [0, n) of the bounce's half of the ping-pong buffer with `threads`
        /// workers over interleaved 4096-ray chunks. Returns the worst per-ray status.</summary>
        public static int Trace(TraceBuffers S, uint[] rays, int n, int bounce, float farPlane, int width, int height,
                                uint[] info, int threads)
        {
            int baseIndex = (bounce % 2 == 1) ? width * height : 0;
            const int Chunk = 4096;
            int chunks = (n + Chunk - 1) / Chunk, worst = 0;
            object gate = new object();
            Parallel.For(0, chunks, new ParallelOptions { MaxDegreeOfParallelism = Math.Max(1, threads) }, c =>
            {
                int w = 0;
                for (int i = c * Chunk; i < Math.Min(n, (c + 1) * Chunk); i++)
                    w = Math.Max(w, TraceRay(S, rays, baseIndex + i, bounce, farPlane, width, height, info));
                lock (gate) worst = Math.Max(worst, w);
            });
            return worst;
        }

        static T[] Load<T>(string dir, string name) where T : struct =>
            MemoryMarshal.Cast<byte, T>(File.ReadAllBytes(Path.Combine(dir, name))).ToArray();

        public static int Main(string[] args)
        {
            if (args.Length < 1) { Console.Error.WriteLine("usage: ScalarTraversal <dump dir> [threads]"); return 2; }
            string dir = args[0];
            int threads = args.Length > 1 ? int.Parse(args[1]) : Environment.ProcessorCount;
            var S = new TraceBuffers { Nodes = Load<uint>(dir, "nodes.bin"), Tris = Load<uint>(dir, "tris.bin"),
                                       Tlas = Load<int>(dir, "tlas.bin"), MeshData = Load<uint>(dir, "meshdata.bin"),
                                       Materials = Load<uint>(dir, "materials.bin") };
            string[] p = File.ReadAllText(Path.Combine(dir, "params.txt")).Split((char[])null, StringSplitOptions.RemoveEmptyEntries);
            int n = int.Parse(p[0]), bounce = int.Parse(p[1]), W = int.Parse(p[3]), H = int.Parse(p[4]);
            float far = float.Parse(p[2], System.Globalization.CultureInfo.InvariantCulture);
            uint[] pristine = Load<uint>(dir, "rays.bin"), expected = Load<uint>(dir, "expected_hits.bin");
            uint[] rays = (uint[])pristine.Clone();
            Trace(S, rays, n, bounce, far, W, H, null, threads);  // warm-up
            int reps = 0;
            var sw = Stopwatch.StartNew();
            do { Array.Copy(pristine, rays, rays.Length); Trace(S, rays, n, bounce, far, W, H, null, threads); reps++; }
            while (sw.Elapsed.TotalSeconds < 10.0);
            double secs = sw.Elapsed.TotalSeconds;
            int baseIndex = (bounce % 2 == 1) ? W * H : 0, bad = 0;
            for (int i = 0; i < n; i++)
                for (int k = 0; k < 4; k++)
                    if (rays[(baseIndex + i) * 12 + 8 + k] != expected[i * 4 + k]) { bad++; break; }
            Console.WriteLine($"{{\"csharp_scalar_mrays_s\": {n * (double)reps / secs / 1e6:F3}, \"threads\": {threads}, " +
                              $"\"rays\": {n}, \"reps\": {reps}, \"mismatches\": {bad}}}");
            return bad == 0 ? 0 : 1;
        }
    }
}
