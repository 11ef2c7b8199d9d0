"""Generates sep_ko.hip: the register-A separable-conv kernel (csrc/sepconv.hip) with knock-out
variants for timing decomposition (KO bit 1: no MFMA, 2: depthwise = centre tap only, 4: no global
loads inside the k-loop, 8: no barrier in the k-loop, 16: no y store,
32: no z store).  Lab only; results are not meaningful."""
import re, sys
src = open(sys.argv[1]).read()
a = src.index('// ------------------------------------------------------------------------------------------\n// Register-A schedule.')
b = src.index('template <int MODE, bool DROP, int BN>\nvoid launch_rk_t')
k = src[a:b]
k = k.replace('template <int MODE, bool DROP, int EPI, int BN, bool WRITE_Y>\n__global__ __launch_bounds__(256, 2) void sepconv_rk_kernel(',
              'template <int MODE, bool DROP, int EPI, int BN, bool WRITE_Y, int KO>\n__global__ __launch_bounds__(256, 2) void sepconv_ko_kernel(')
k = k.replace('constexpr int RX = BK + 4;', '').replace('constexpr int HPIX = HHp * HWp;            // 180 halo pixels', '')
k = k.replace('                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bf.x, acc[tn], 0, 0, 0);\n',
              '                if constexpr (!(KO & 1)) {\n                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bf.x, acc[tn], 0, 0, 0);\n')
k = k.replace('                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bf.w, acc[tn], 0, 0, 0);\n',
              '                acc[tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bf.w, acc[tn], 0, 0, 0);\n                } else { acc[tn][0] += a.x * bf.x + a.w * bf.w; }\n')
k = k.replace('            for (int dy = 0; dy < 3; ++dy)\n#pragma unroll\n                for (int dx = 0; dx < 3; ++dx) {',
              '            for (int dy = (KO & 2) ? 1 : 0; dy < ((KO & 2) ? 2 : 3); ++dy)\n#pragma unroll\n                for (int dx = (KO & 2) ? 1 : 0; dx < ((KO & 2) ? 2 : 3); ++dx) {')
k = k.replace('        load_halo((kt + 1) * BK);\n        load_b((kt + 1) * BK);\n',
              '        if constexpr (!(KO & 4)) {\n        load_halo((kt + 1) * BK);\n        load_b((kt + 1) * BK);\n        }\n')
k = k.replace('            store_b(buf ^ 1);\n        }\n        __syncthreads();\n',
              '            store_b(buf ^ 1);\n        }\n        if constexpr (!(KO & 8)) __syncthreads();\n')
k = k.replace('        if constexpr (WRITE_Y) {  // y for', '        if constexpr (WRITE_Y && !(KO & 16)) {  // y for')
k = k.replace('        if (col >= g.Cout) continue;\n#pragma unroll\n        for (int r = 0; r < 16; ++r) {\n            const int p = wave * 32',
              '        if (col >= g.Cout || (KO & 32)) continue;\n#pragma unroll\n        for (int r = 0; r < 16; ++r) {\n            const int p = wave * 32')
k = k.replace('    const int nk = (Cin + BK - 1) / BK;\n    load_halo(0);', '    const int nk = (KO & 64) ? 1 : (Cin + BK - 1) / BK;\n    load_halo(0);')
out = '#include "sepconv.h"\nnamespace unet {\nnamespace sep {\nnamespace {\n' + k + '}\n}\n}\n'
open(sys.argv[2], 'w').write(out)
