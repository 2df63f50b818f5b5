/*
 * oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's
 * Selection + Projection semantics (ariesdevil/datafusion v0.5.1,
 * src/execution/{expression,filter,projection}.rs + arrow 0.12 array_ops).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline. The product path
 * (datafusion_amd, libdfmi.so) never links or calls it.
 *
 * Parity pinning: the restatement is checked against every known-answer
 * fixture the reference tree holds for this path (tests/golden/).
 * Semantics the reference's own files do not pin (null ordering, divide by
 * zero, integer overflow, NaN, Int64 gather, Utf8 equality) are the arrow
 * 0.12.x rules restated — "parity unpinned (arrow 0.12.x semantics restated)".
 */
#ifndef DF_ORACLE_H
#define DF_ORACLE_H

#include "../include/dfmi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_result oracle_result;

/* ProjectRelation(FilterRelation(batch)) evaluated the reference's way.
 * pred_nodes == NULL: no Selection. num_projections == 0: no Projection
 * (FilterRelation output). Projection i is proj_nodes[i][0 .. proj_lens[i]).
 * Compile errors and run-time errors are both reported through err, in the
 * order the reference raises them. `input` holds host pointers. */
int32_t oracle_filter_project(const dfmi_expr_node* pred_nodes, int32_t pred_len,
                              const dfmi_expr_node* const* proj_nodes, const int32_t* proj_lens,
                              int32_t num_projections, const dfmi_schema* schema,
                              const dfmi_batch* input, uint32_t flags,
                              oracle_result** out, dfmi_error* err);

/* Same, but feeding the input through the pull pipeline in batches of
 * batch_rows (the csv::Reader batch size, csv_sql.rs:49). Returns only the
 * total output row count (the CPU baseline timing loop). */
int32_t oracle_run_batched(const dfmi_expr_node* pred_nodes, int32_t pred_len,
                           const dfmi_expr_node* const* proj_nodes, const int32_t* proj_lens,
                           int32_t num_projections, const dfmi_schema* schema,
                           const dfmi_batch* input, int64_t batch_rows, uint32_t flags,
                           int64_t* out_rows, dfmi_error* err);

int32_t oracle_result_num_columns(const oracle_result* r);
/* Host view of result column i (validity NULL when null_count == 0). */
int32_t oracle_result_column(const oracle_result* r, int32_t i, dfmi_column* view,
                             const char** name);
void oracle_result_free(oracle_result* r);

/* compile_scalar_expr name/type only (RuntimeExpr::get_name/get_type). */
int32_t oracle_compile_info(const dfmi_expr_node* nodes, int32_t n, const dfmi_schema* schema,
                            uint32_t flags, char* name, int64_t name_cap, int32_t* type,
                            dfmi_error* err);

/* Aggregate extension (DFMI_FLAG_EXT_AGGREGATE): Aggregate(Selection?(scan))
 * with no GROUP BY over `input` pulled in batches of batch_rows (<= 0: one
 * batch); aggregate j is names[j](arg j) with the planner's return type. */
int32_t oracle_aggregate(const dfmi_expr_node* pred_nodes, int32_t pred_len, const char* const* names,
                         const dfmi_expr_node* const* arg_nodes, const int32_t* arg_lens,
                         const int32_t* return_types, int32_t num_aggs, const dfmi_schema* schema,
                         const dfmi_batch* input, int64_t batch_rows, uint32_t flags, dfmi_agg_value* out,
                         dfmi_error* err);
/* GROUP BY extension: one key (Boolean, integer, float -- totalOrder, one
 * group per bit pattern --, Utf8 -- bytewise, the keys' bytes into
 * key_offsets / key_data); groups in key order, null last. */
int32_t oracle_aggregate_grouped_multi(const dfmi_expr_node* pred_nodes, int32_t pred_len,
                                       const dfmi_expr_node* const* key_nodes, const int32_t* key_lens, int32_t nkeys,
                                       const char* const* names, const dfmi_expr_node* const* arg_nodes,
                                       const int32_t* arg_lens, const int32_t* return_types, int32_t n,
                                       const dfmi_schema* schema, const dfmi_batch* input, int64_t batch_rows,
                                       uint32_t flags, int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* out,
                                       int64_t* num_groups, int32_t key_part, int32_t* key_offsets, uint8_t* key_data,
                                       int64_t key_data_cap, dfmi_error* err);
int32_t oracle_aggregate_grouped(const dfmi_expr_node* pred_nodes, int32_t pred_len, const dfmi_expr_node* key_nodes,
                                 int32_t key_len, const char* const* names, const dfmi_expr_node* const* arg_nodes,
                                 const int32_t* arg_lens, const int32_t* return_types, int32_t n,
                                 const dfmi_schema* schema, const dfmi_batch* input, int64_t batch_rows,
                                 uint32_t flags, int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* out,
                                 int64_t* num_groups, int32_t* key_offsets, uint8_t* key_data, int64_t key_data_cap,
                                 dfmi_error* err);

/* Synthetic tables, bit-identical to the device generator. */
uint64_t oracle_splitmix64(uint64_t x);
void oracle_gen_unit_f64(uint64_t seed, uint32_t col, int64_t row0, int64_t n, double* out);
void oracle_gen_i64(uint64_t seed, uint32_t col, int64_t row0, int64_t n, int64_t lo, int64_t hi,
                    int64_t* out);

#ifdef __cplusplus
}
#endif
#endif
