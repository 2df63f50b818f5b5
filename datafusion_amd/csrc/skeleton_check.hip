// Build-time check of jit_skeleton.hip: instantiates every skeleton template
// with a representative generated body (one Float64 predicate, a gathered
// column, a Utf8 gather, integer division at several widths), so a broken skeleton fails `make` rather than the
// first query compile on the GPU. Not linked into libdfmi.so.
#include <hip/hip_runtime.h>

#include "jit_skeleton.hip"

extern "C" __global__ __launch_bounds__(512) void dfmi_skeleton_check(const dfmi::Args A) {
    constexpr int BLOCK = 512, K = 8, WAVES = BLOCK / 64, NCH = 2;
    const int tid = threadIdx.x, lane = tid & 63, wave = dfmi::uni(tid >> 6);
    __shared__ dfmi::Tile<BLOCK, K, NCH> T;
    __shared__ dfmi::Utf8Stage<> G[WAVES];
    const unsigned tile = blockIdx.x;
    const i64 base = (i64)tile * (BLOCK * K);
    const i64 rem = A.n_rows - base;
    u64 c0[K];
    for (int k = 0; k < K; ++k) c0[k] = (k * BLOCK + tid < rem) ? ((const u64*)A.col[0] + base)[k * BLOCK + tid] : 0ull;
    unsigned selm = 0;
    for (int k = 0; k < K; ++k) {
        const i64 row = base + k * BLOCK + tid;
        selm |= (unsigned)(row < A.n_rows && dfmi::f64(c0[k]) > dfmi::f64(A.lits[0])) << k;
    }
    unsigned cnt[NCH][K];
    u64 wm[K];
    int us[K], ue[K];
    bool eq[K];
    dfmi::utf8_offs_tile<BLOCK, K>(A, 0, base, lane, wave, ~0u, us, ue);
    dfmi::utf8_eq_lit_tile<BLOCK, K>(A, 0, 0, A.str + A.str_off[0], us, ue, lane, eq);
    bool eq2[K];
    dfmi::utf8_eq_lit_tile_reg<BLOCK, K, 4>(A, 0, 0, A.str + A.str_off[0], us, ue, lane, eq2);
    for (int k = 0; k < K; ++k) eq[k] = eq[k] || eq2[k];
    for (int k = 0; k < K; ++k) {
        selm |= (unsigned)eq[k] << k;
        wm[k] = __ballot((selm >> k) & 1);
        cnt[0][k] = (selm >> k) & 1;
        cnt[1][k] = ((selm >> k) & 1) ? (unsigned)(dfmi::utf8_end(us[k], ue[k], lane) - us[k]) : 0u;
    }
    dfmi::tile_offsets<BLOCK, K, NCH, 4, 2, 16>(A, T, tile, cnt, lane, wave);
    const i64 obase = (i64)T.prefix[0];
    unsigned dst[K];
    for (int k = 0; k < K; ++k) dst[k] = (unsigned)T.excl[0][k * WAVES + wave] + dfmi::lane_rank(wm[k]);
    for (int k = 0; k < K; ++k)
        if ((selm >> k) & 1) ((u64*)A.out[0] + obase)[dst[k]] = c0[k];
    dfmi::utf8_gather<BLOCK, K, NCH, dfmi::kStageChunks>(A, T, 1, 0, 1, selm, wm, dst, us, ue, G[wave], lane, wave);
    dfmi::utf8_gather_serial<BLOCK, K, NCH, dfmi::kStageChunks>(A, T, 1, 0, 1, selm, wm, dst, us, ue, G[wave], lane, wave);
    dfmi::utf8_gather_lane<BLOCK, K, NCH>(A, T, 1, 0, 1, selm, dst, us, ue, lane, wave);
    dfmi::utf8_offsets_src<BLOCK, K, NCH>(A, T, 1, 1, selm, wm, dst, us, ue, lane, wave);
    const bool b = dfmi::cmp_opt<2>(true, false, false) && dfmi::utf8_eq_lit(A, 0, base, 0, A.str) &&
                   dfmi::utf8_eq_col(A, 0, 1, base) && dfmi::utf8_valid(A, 0, base);
    if (b) dfmi::report_err(A.err, 1, base, dfmi::ERRK_DIV_ZERO);
    if (tid == 0 && dfmi::bitmap_word(A.valid[0], 0, A.n_rows) == 7)
        A.totals[0] = (u64)dfmi::idiv<i64>((i64)A.lits[1], (i64)A.lits[2]) +
                      (u64)dfmi::idiv<i8>((i8)A.lits[1], dfmi::int_min<i8>()) + dfmi::idiv<u16>((u16)A.lits[1], 3);
}
