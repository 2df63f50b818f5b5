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

/* ---------------------------------------------------------------------------
 * CSV source: CsvDataSource::new(schema, csv::Reader::new(file, schema,
 * has_header, batch_size, None)) (datasource.rs:31-50, csv_sql.rs:49), native.
 * Batches come back as HOST columns in pinned memory (ready for
 * dfmi_filter_project_host's direct DMA); they stay valid until the next
 * dfmi_csv_next or dfmi_csv_close. The reader parses batch i+1 (host threads)
 * while the caller works on batch i. `threads` <= 0: up to 8.
 * Errors: IoError (open) as DFMI_ERR_GENERAL "IoError: ...", a field that does
 * not parse as ArrowError(ParseError) "Error while parsing value <field>".
 * ------------------------------------------------------------------------- */
typedef struct dfmi_csv_reader dfmi_csv_reader;

int32_t dfmi_csv_open(const char* path, const dfmi_schema* schema, int32_t has_header, int64_t batch_size,
                      int32_t threads, dfmi_csv_reader** out, dfmi_error* err);
/* *has_batch = 0 at the end of the file. */
int32_t dfmi_csv_next(dfmi_csv_reader* reader, dfmi_batch* out, int32_t* has_batch, dfmi_error* err);
int64_t dfmi_csv_num_records(const dfmi_csv_reader* reader);
void dfmi_csv_close(dfmi_csv_reader* reader);

#ifdef __cplusplus
}
#endif
#endif
