/*
 * isa_probe.hip — issue cost of the instruction kinds the simulation kernel is made of,
 * measured on the GPU (gfx950): every wave runs `iters` iterations of a block of 32
 * independent instructions of one kind; the grid holds `waves_per_simd` waves on every
 * SIMD, so the time per instruction per SIMD is the kind's issue cost with the pipeline
 * kept full by the other waves.
 *
 *   hipcc --offload-arch=gfx950 -O3 tools/isa_probe.hip -o build/isa_probe
 *   build/isa_probe [waves_per_simd]
 *
 * Diagnostic tool only; nothing in the product uses it.
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define REP4(x) x x x x
#define REP32(x) REP4(REP4(x)) REP4(x) REP4(x) REP4(x) REP4(x)

#define PROBE(name, body)                                                         \
    __global__ void __launch_bounds__(256) name(double* out, int iters) {          \
        double a = threadIdx.x * 1e-3, b = 1.000001, c = 0.5, d = 0.25, e = 0.125;           \
        uint32_t u = threadIdx.x, w = 7;                                           \
        for (int i = 0; i < iters; ++i) {                                          \
            body                                                                   \
        }                                                                          \
        if (a == 12345.0 && u == 77u) out[0] = a + b + c + d + e + (double)w;          \
    }

/* 32 instructions per iteration, spread over independent registers (4 chains) */
PROBE(p_add_f64, REP4(asm volatile("v_add_f64 %0, %0, %1\n v_add_f64 %2, %2, %1\n v_add_f64 %3, %3, %1\n v_add_f64 %4, %4, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %2, %2, %1\n v_add_f64 %3, %3, %1\n v_add_f64 %4, %4, %1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e));))
PROBE(p_fma_f64, REP4(asm volatile("v_fma_f64 %0, %0, %1, %1\n v_fma_f64 %2, %2, %1, %1\n v_fma_f64 %3, %3, %1, %1\n v_fma_f64 %4, %4, %1, %1\n v_fma_f64 %0, %0, %1, %1\n v_fma_f64 %2, %2, %1, %1\n v_fma_f64 %3, %3, %1, %1\n v_fma_f64 %4, %4, %1, %1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e));))
PROBE(p_mov_b32, REP4(asm volatile("v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, %0" :: "v"(u) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");))
PROBE(p_mov_b64, REP4(asm volatile("v_mov_b64 v[40:41], %0\n v_mov_b64 v[42:43], %0\n v_mov_b64 v[44:45], %0\n v_mov_b64 v[46:47], %0\n v_mov_b64 v[48:49], %0\n v_mov_b64 v[50:51], %0\n v_mov_b64 v[52:53], %0\n v_mov_b64 v[54:55], %0" :: "v"(a) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");))
PROBE(p_add_u32, REP4(asm volatile("v_add_u32 v40, %0, v40\n v_add_u32 v41, %0, v41\n v_add_u32 v42, %0, v42\n v_add_u32 v43, %0, v43\n v_add_u32 v44, %0, v44\n v_add_u32 v45, %0, v45\n v_add_u32 v46, %0, v46\n v_add_u32 v47, %0, v47" :: "v"(u) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");))
PROBE(p_cndmask, REP4(asm volatile("v_cndmask_b32 v40, %0, v40, vcc\n v_cndmask_b32 v41, %0, v41, vcc\n v_cndmask_b32 v42, %0, v42, vcc\n v_cndmask_b32 v43, %0, v43, vcc\n v_cndmask_b32 v44, %0, v44, vcc\n v_cndmask_b32 v45, %0, v45, vcc\n v_cndmask_b32 v46, %0, v46, vcc\n v_cndmask_b32 v47, %0, v47, vcc" :: "v"(u) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");))
PROBE(p_dpp, REP4(asm volatile("v_mov_b32_dpp v40, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v41, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v42, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v43, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v44, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v45, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v46, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v47, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" :: "v"(u) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");))
PROBE(p_readlane, REP4(asm volatile("v_readlane_b32 s40, %0, 3\n v_readlane_b32 s41, %0, 5\n v_readlane_b32 s42, %0, 7\n v_readlane_b32 s43, %0, 9\n v_readlane_b32 s44, %0, 11\n v_readlane_b32 s45, %0, 13\n v_readlane_b32 s46, %0, 15\n v_readlane_b32 s47, %0, 17" :: "v"(u) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");))
PROBE(p_writelane, REP4(asm volatile("v_writelane_b32 v40, %0, 3\n v_writelane_b32 v41, %0, 5\n v_writelane_b32 v42, %0, 7\n v_writelane_b32 v43, %0, 9\n v_writelane_b32 v44, %0, 11\n v_writelane_b32 v45, %0, 13\n v_writelane_b32 v46, %0, 15\n v_writelane_b32 v47, %0, 17" :: "s"(w) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");))
PROBE(p_readlane_use, REP4(asm volatile("v_readlane_b32 s40, %0, 3\n s_add_u32 s48, s40, 1\n v_readlane_b32 s41, %0, 5\n s_add_u32 s49, s41, 1\n v_readlane_b32 s42, %0, 7\n s_add_u32 s50, s42, 1\n v_readlane_b32 s43, %0, 9\n s_add_u32 s51, s43, 1" :: "v"(u) : "s40", "s41", "s42", "s43", "s48", "s49", "s50", "s51", "scc");))
PROBE(p_salu, REP4(asm volatile("s_add_u32 s40, s40, %0\n s_add_u32 s41, s41, %0\n s_add_u32 s42, s42, %0\n s_add_u32 s43, s43, %0\n s_add_u32 s44, s44, %0\n s_add_u32 s45, s45, %0\n s_add_u32 s46, s46, %0\n s_add_u32 s47, s47, %0" :: "s"(w) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "scc");))
PROBE(p_mixed_f64_salu, REP4(asm volatile("v_add_f64 %0, %0, %1\n s_add_u32 s40, s40, 1\n v_add_f64 %2, %2, %1\n s_add_u32 s41, s41, 1\n v_add_f64 %3, %3, %1\n s_add_u32 s42, s42, 1\n v_add_f64 %4, %4, %1\n s_add_u32 s43, s43, 1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e) :: "s40", "s41", "s42", "s43", "scc");))
PROBE(p_cmp_f64, REP4(asm volatile("v_cmp_lt_f64 s[40:41], %0, %1\n v_cmp_lt_f64 s[42:43], %0, %1\n v_cmp_lt_f64 s[44:45], %0, %1\n v_cmp_lt_f64 s[46:47], %0, %1\n v_cmp_lt_f64 s[48:49], %0, %1\n v_cmp_lt_f64 s[50:51], %0, %1\n v_cmp_lt_f64 s[52:53], %0, %1\n v_cmp_lt_f64 s[54:55], %0, %1" :: "v"(a), "v"(b) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");))

PROBE(p_cndmask_s, REP4(asm volatile("v_cndmask_b32_e64 v40, %0, v40, s[40:41]\n v_cndmask_b32_e64 v41, %0, v41, s[40:41]\n v_cndmask_b32_e64 v42, %0, v42, s[40:41]\n v_cndmask_b32_e64 v43, %0, v43, s[40:41]\n v_cndmask_b32_e64 v44, %0, v44, s[40:41]\n v_cndmask_b32_e64 v45, %0, v45, s[40:41]\n v_cndmask_b32_e64 v46, %0, v46, s[40:41]\n v_cndmask_b32_e64 v47, %0, v47, s[40:41]" :: "v"(u) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");))
PROBE(p_cmp_cndmask, REP4(asm volatile("v_cmp_gt_u32 vcc, %0, v40\n v_cndmask_b32 v40, %0, v40, vcc\n v_cmp_gt_u32 vcc, %0, v41\n v_cndmask_b32 v41, %0, v41, vcc\n v_cmp_gt_u32 vcc, %0, v42\n v_cndmask_b32 v42, %0, v42, vcc\n v_cmp_gt_u32 vcc, %0, v43\n v_cndmask_b32 v43, %0, v43, vcc" :: "v"(u) : "v40", "v41", "v42", "v43", "vcc");))
PROBE(p_cmp_cndmask_s, REP4(asm volatile("v_cmp_gt_u32_e64 s[40:41], %0, v40\n v_cndmask_b32_e64 v40, %0, v40, s[40:41]\n v_cmp_gt_u32_e64 s[42:43], %0, v41\n v_cndmask_b32_e64 v41, %0, v41, s[42:43]\n v_cmp_gt_u32_e64 s[44:45], %0, v42\n v_cndmask_b32_e64 v42, %0, v42, s[44:45]\n v_cmp_gt_u32_e64 s[46:47], %0, v43\n v_cndmask_b32_e64 v43, %0, v43, s[46:47]" :: "v"(u) : "v40", "v41", "v42", "v43", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");))
PROBE(p_mul_f64, REP4(asm volatile("v_mul_f64 %0, %0, %1\n v_mul_f64 %2, %2, %1\n v_mul_f64 %3, %3, %1\n v_mul_f64 %4, %4, %1\n v_mul_f64 %0, %0, %1\n v_mul_f64 %2, %2, %1\n v_mul_f64 %3, %3, %1\n v_mul_f64 %4, %4, %1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e));))
PROBE(p_ds_read, REP4(asm volatile("ds_read_b64 v[40:41], %0\n ds_read_b64 v[42:43], %0 offset:8\n ds_read_b64 v[44:45], %0 offset:16\n ds_read_b64 v[46:47], %0 offset:24\n ds_read_b64 v[48:49], %0 offset:32\n ds_read_b64 v[50:51], %0 offset:40\n ds_read_b64 v[52:53], %0 offset:48\n ds_read_b64 v[54:55], %0 offset:56\n s_waitcnt lgkmcnt(0)" :: "v"(u * 8u & 0x3ff8u) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");))
PROBE(p_lshl_add_u64, REP4(asm volatile("v_lshl_add_u64 v[40:41], %0, 3, v[40:41]\n v_lshl_add_u64 v[42:43], %0, 3, v[42:43]\n v_lshl_add_u64 v[44:45], %0, 3, v[44:45]\n v_lshl_add_u64 v[46:47], %0, 3, v[46:47]\n v_lshl_add_u64 v[48:49], %0, 3, v[48:49]\n v_lshl_add_u64 v[50:51], %0, 3, v[50:51]\n v_lshl_add_u64 v[52:53], %0, 3, v[52:53]\n v_lshl_add_u64 v[54:55], %0, 3, v[54:55]" :: "v"(a) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");))
PROBE(p_pk_mov, REP4(asm volatile("v_pk_mov_b32 v[40:41], %0, %0 op_sel:[0,1]\n v_pk_mov_b32 v[42:43], %0, %0 op_sel:[0,1]\n v_pk_mov_b32 v[44:45], %0, %0 op_sel:[0,1]\n v_pk_mov_b32 v[46:47], %0, %0 op_sel:[0,1]\n v_pk_mov_b32 v[48:49], %0, %0 op_sel:[0,1]\n v_pk_mov_b32 v[50:51], %0, %0 op_sel:[0,1]\n v_pk_mov_b32 v[52:53], %0, %0 op_sel:[0,1]\n v_pk_mov_b32 v[54:55], %0, %0 op_sel:[0,1]" :: "v"(a) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");))
PROBE(p_sqrt_f64, REP4(asm volatile("v_sqrt_f64 %0, %0\n v_sqrt_f64 %2, %2\n v_sqrt_f64 %3, %3\n v_sqrt_f64 %4, %4\n v_sqrt_f64 %0, %0\n v_sqrt_f64 %2, %2\n v_sqrt_f64 %3, %3\n v_sqrt_f64 %4, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e));))
PROBE(p_rcp_f64, REP4(asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n v_rcp_f64 %4, %4\n v_rcp_f64 %0, %0\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n v_rcp_f64 %4, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e));))
PROBE(p_snop, REP4(asm volatile("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0");))

struct Probe {
    const char* name;
    void (*fn)(double*, int);
};

int main(int argc, char** argv) {
    const int wps = argc > 1 ? atoi(argv[1]) : 5;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    double* out = nullptr;
    hipMalloc(&out, 64);
    const Probe probes[] = {{"v_add_f64", p_add_f64},     {"v_fma_f64", p_fma_f64},   {"v_mov_b32", p_mov_b32},
                            {"v_mov_b64", p_mov_b64},     {"v_add_u32", p_add_u32},   {"v_cndmask_b32", p_cndmask},
                            {"v_mov_b32_dpp", p_dpp},     {"v_readlane_b32", p_readlane}, {"v_writelane_b32", p_writelane},
                            {"readlane+salu_use (pairs)", p_readlane_use}, {"s_add_u32", p_salu},
                            {"v_add_f64+s_add (pairs)", p_mixed_f64_salu}, {"v_cmp_lt_f64", p_cmp_f64},
                            {"v_cndmask_b32_e64 sgpr mask", p_cndmask_s}, {"v_cmp vcc + v_cndmask (pairs)", p_cmp_cndmask},
                            {"v_cmp sgpr + v_cndmask (pairs)", p_cmp_cndmask_s}, {"v_mul_f64", p_mul_f64},
                            {"ds_read_b64 (8 + waitcnt)", p_ds_read}, {"v_lshl_add_u64", p_lshl_add_u64}, {"v_pk_mov_b32", p_pk_mov},
                            {"v_sqrt_f64", p_sqrt_f64}, {"v_rcp_f64", p_rcp_f64}, {"s_nop 0", p_snop}};
    const int iters = 20000;
    /* 4 waves per block (one per SIMD), wps blocks per CU */
    const int blocks = cus * wps;
    std::printf("{\"cus\": %d, \"clock_khz\": %d, \"waves_per_simd\": %d, \"results\": [\n", cus, clk_khz, wps);
    for (size_t k = 0; k < sizeof(probes) / sizeof(probes[0]); ++k) {
        hipLaunchKernelGGL(probes[k].fn, dim3(blocks), dim3(256), 0, 0, out, 10);
        hipDeviceSynchronize();
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        hipLaunchKernelGGL(probes[k].fn, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        /* instructions per SIMD = waves per SIMD x iters x 32 */
        const double per_simd = (double)wps * iters * 32.0;
        const double ns_per = ms * 1e6 / per_simd;
        std::printf("  {\"kind\": \"%s\", \"ms\": %.3f, \"ns_per_wave_instr_per_simd\": %.4f, \"cycles_at_2.4GHz\": %.2f}%s\n",
                    probes[k].name, ms, ns_per, ns_per * 2.4, k + 1 < sizeof(probes) / sizeof(probes[0]) ? "," : "");
    }
    std::printf("]}\n");
    return 0;
}
