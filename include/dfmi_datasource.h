/*
 * dfmi_datasource.h — synthetic table source on the device (bench inputs).
 *
 * Plugs in where the reference's DataSource trait sits
 * (src/execution/datasource.rs:26-29): it fills HBM-resident columns of the
 * seeded synthetic tables of SURVEY.md §8d directly on the GPU, bit-identical
 * to the CPU oracle's generator (oracle/df_oracle.cpp oracle_gen_*), so a
 * 1e9-row table never crosses PCIe.
 *   value(seed, col, row) = splitmix64(splitmix64(seed + col*0xD1B54A32D192ED03) ^ row)
 *   UNIT_F64: (value >> 11) * 2^-53            in [0, 1)
 *   I64:      lo + value % (hi - lo)           in [lo, hi)
 */
#ifndef DFMI_DATASOURCE_H
#define DFMI_DATASOURCE_H
#include "dfmi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum dfmi_gen_kind { DFMI_GEN_UNIT_F64 = 1, DFMI_GEN_I64 = 2 } dfmi_gen_kind;

/* Fill out[0..n) (device pointer) with rows row0 .. row0+n of column `col`.
 * Asynchronous on the context's stream. */
int32_t dfmi_generate_column(dfmi_context* ctx, int32_t kind, uint64_t seed, uint32_t col,
                             int64_t row0, int64_t n, int64_t lo, int64_t hi, void* out,
                             dfmi_error* err);

#ifdef __cplusplus
}
#endif
#endif
