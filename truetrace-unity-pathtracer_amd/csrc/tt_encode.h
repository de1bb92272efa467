// tt_encode.h — the colour encodings the any-hit kernel's radiance-cache path writes (row f1,
// IntersectionKernels.compute:456-485 with RadianceCache on, GlobalDefines.cginc:15):
// packRGBE / unpackRGBE (CommonData.cginc:479-509) and EncodeRGB / DecodeRGB (:1576-1619), plus
// HLSL pow as D3D lowers it (exp2(y * log2(x)), float intermediates).
//
// The reference leaves log2 / exp2 precision to the D3D driver. Pinned here (and restated in
// oracle/tt_oracle.c): log2f / exp2f are evaluated in double precision with the fixed series below
// (frexp / ldexp for the exponent, IEEE + - * / only, no contraction) and rounded once to float --
// i.e. correctly rounded except in cases too close to a rounding boundary for a 1e-16 relative
// error, where both sides still agree bit for bit. floor(log2(x)) in packRGBE and pow(2, n) for an
// integer n are exact (frexp / ldexp), as the refit pins its pow2(ceil(log2)). round() is
// round-half-to-even (DXIL round_ne); float -> uint is D3D's (NaN -> 0, saturating); min/max are
// IEEE minNum / maxNum; mul(M, c) rows are fmaf(m2, z, fmaf(m1, y, m0 * x)); HLSL's unsuffixed
// literals are taken as doubles rounded to float.
#ifndef TT_ENCODE_H
#define TT_ENCODE_H
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tt_enc {

__device__ __forceinline__ float log2f_pinned(float xf) {
    if (xf != xf || xf < 0.0f) return __int_as_float(0x7fc00000);
    if (xf == 0.0f) return -__builtin_inff();
    if (xf == __builtin_inff()) return xf;
    int e;
    double m = frexp((double)xf, &e);  // xf = m * 2^e, m in [0.5, 1)
    if (m < 0.70710678118654752) {
        m = m * 2.0;
        e = e - 1;
    }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double p = 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    p = p * s2 + 1.0;
    const double ln_m = 2.0 * s * p;
    return (float)((double)e + ln_m * 1.4426950408889634);
}

__device__ __forceinline__ float exp2f_pinned(float yf) {
    if (yf != yf) return yf;
    if (yf >= 128.0f) return __builtin_inff();
    if (yf < -160.0f) return 0.0f;
    const double y = (double)yf, k = floor(y), f = y - k;  // exact: yf has 24 significant bits
    const double r = f * 0.69314718055994531;
    double t = 1.0, sum = 1.0;
    for (int n = 1; n <= 22; n++) {
        t = t * r / (double)n;
        sum = sum + t;
    }
    return (float)ldexp(sum, (int)k);
}

// HLSL pow(x, y) = exp2(y * log2(x)) with float intermediates
__device__ __forceinline__ float pow_pinned(float x, float y) { return exp2f_pinned(y * log2f_pinned(x)); }

__device__ __forceinline__ uint32_t ftou(float f) {  // D3D float -> uint
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}
__device__ __forceinline__ float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }
__device__ __forceinline__ float mulrow(float m0, float m1, float m2, float x, float y, float z) {
    return __builtin_fmaf(m2, z, __builtin_fmaf(m1, y, m0 * x));
}

// packRGBE — CommonData.cginc:479-496
__device__ __forceinline__ uint32_t packRGBE(float r, float g, float b) {
    const float va[3] = {fmaxf(0.0f, r), fmaxf(0.0f, g), fmaxf(0.0f, b)};
    const float max_abs = fmaxf(va[0], fmaxf(va[1], va[2]));
    if (max_abs == 0.0f) return 0u;
    int e;
    (void)frexpf(max_abs, &e);
    const float exponent = (float)(e - 1);  // floor(log2(max_abs)), exact
    uint32_t result = ftou(clampf(exponent + 20.0f, 0.0f, 31.0f)) << 27;
    const float scale = exp2f_pinned(-exponent) * 256.0f;
    uint32_t vu[3];
    for (int k = 0; k < 3; k++) vu[k] = ftou(fminf(511.0f, rintf(va[k] * scale)));
    result |= vu[0];
    result |= vu[1] << 9;
    result |= vu[2] << 18;
    return result;
}

// unpackRGBE — CommonData.cginc:498-509
__device__ __forceinline__ float3 unpackRGBE(uint32_t x) {
    const int exponent = (int)(x >> 27) - 20;
    const float scale = exp2f_pinned((float)exponent) / 256.0f;
    return make_float3((float)(x & 0x1ffu) * scale, (float)((x >> 9) & 0x1ffu) * scale,
                       (float)((x >> 18) & 0x1ffu) * scale);
}

// EncodeRGB — CommonData.cginc:1576-1590 (RTXDI_RGBToXYZInRec709, :1555-1563)
__device__ __forceinline__ uint32_t EncodeRGB(float r, float g, float b) {
    const float X = mulrow((float)0.4123907992659595, (float)0.3575843393838780, (float)0.1804807884018343, r, g, b);
    const float Y = mulrow((float)0.2126390058715104, (float)0.7151686787677559, (float)0.0721923153607337, r, g, b);
    const float Z = mulrow((float)0.0193308187155918, (float)0.1191947797946259, (float)0.9505321522496608, r, g, b);
    const float logY = (float)409.6 * (log2f_pinned(Y) + 20.0f);
    const uint32_t Le = ftou(clampf(logY, 0.0f, 16383.0f));
    if (Le == 0u) return 0u;
    const float invDenom = 1.0f / ((-2.0f * X + 12.0f * Y) + 3.0f * ((X + Y) + Z));
    const float u = (4.0f * X) * invDenom, v = (9.0f * Y) * invDenom;
    const uint32_t ue = ftou(clampf(820.0f * u, 0.0f, 511.0f)), ve = ftou(clampf(820.0f * v, 0.0f, 511.0f));
    return (Le << 18) | (ue << 9) | ve;
}

// DecodeRGB — CommonData.cginc:1592-1619 (RTXDI_XYZToRGBInRec709, :1564-1574)
__device__ __forceinline__ float3 DecodeRGB(uint32_t packed) {
    const uint32_t Le = packed >> 18;
    if (Le == 0u) return make_float3(0.0f, 0.0f, 0.0f);
    const float logY = ((float)Le + 0.5f) / (float)409.6 - 20.0f;
    const float Y = pow_pinned(2.0f, logY);
    const float u = ((float)((packed >> 9) & 0x1ffu) + 0.5f) / 820.0f;
    const float v = ((float)(packed & 0x1ffu) + 0.5f) / 820.0f;
    const float invDenom = 1.0f / ((6.0f * u - 16.0f * v) + 12.0f);
    const float x = (9.0f * u) * invDenom, y = (4.0f * v) * invDenom;
    const float s = Y / y;
    const float X = s * x, Z = s * ((1.0f - x) - y);
    return make_float3(
        fmaxf(mulrow((float)3.240969941904522, (float)-1.537383177570094, (float)-0.4986107602930032, X, Y, Z), 0.0f),
        fmaxf(mulrow((float)-0.9692436362808803, (float)1.875967501507721, (float)0.04155505740717569, X, Y, Z), 0.0f),
        fmaxf(mulrow((float)0.05563007969699373, (float)-0.2039769588889765, (float)1.056971514242878, X, Y, Z), 0.0f));
}

}  // namespace tt_enc
#endif  // TT_ENCODE_H
