/*
 * dfmi.h — C ABI of the MI355X-native Selection + Projection path.
 *
 * This is the drop-in boundary for the only data-parallel path of the reference
 * (ariesdevil/datafusion v0.5.1): expression compilation plus the
 * FilterRelation/ProjectRelation per-batch evaluation in src/execution/.
 * Every entry point names the reference interface it replaces (file:line under
 * the reference tree). No torch or HIP types appear in the signatures: device
 * buffers are plain pointers, streams are opaque `void*` (hipStream_t).
 *
 * Semantics follow the reference bit-for-bit (see DESIGN.md "Semantics"):
 *   - comparisons never produce nulls; null ordering is arrow 0.12's bool_op
 *     (NULL < x is true, NULL = NULL is true, ...);
 *   - math propagates nulls, Float64 rounds once per operator (no FMA);
 *   - a non-null zero divisor is ArrowError(DivideByZero);
 *   - a Selection drops validity and copies raw slot bits of selected rows;
 *   - only Float64 and Utf8 columns can be filtered unless an extension flag
 *     is given (filter.rs:106-110).
 */
#ifndef DFMI_H
#define DFMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version of this header's structs and entry points. 2: dfmi_column.offset
 * (arrow ArrayData::offset), dfmi_abi_version(), the caller-owned output form
 * dfmi_filter_project_host_batches_into. A binding compares the library's
 * dfmi_abi_version() with the constant it was built against. */
#define DFMI_ABI_VERSION 3

/* DFMI_ABI_VERSION of the loaded library. */
int32_t dfmi_abi_version(void);

/* ---------------------------------------------------------------------------
 * Types. Subset of arrow::datatypes::DataType that logicalplan.rs can name
 * (ScalarValue logicalplan.rs:93-108, get_supertype logicalplan.rs:443-551).
 * ------------------------------------------------------------------------- */
typedef enum dfmi_type {
    DFMI_TYPE_NULL = 0, /* ScalarValue::Null only */
    DFMI_TYPE_BOOLEAN = 1,
    DFMI_TYPE_INT8 = 2,
    DFMI_TYPE_INT16 = 3,
    DFMI_TYPE_INT32 = 4,
    DFMI_TYPE_INT64 = 5,
    DFMI_TYPE_UINT8 = 6,
    DFMI_TYPE_UINT16 = 7,
    DFMI_TYPE_UINT32 = 8,
    DFMI_TYPE_UINT64 = 9,
    DFMI_TYPE_FLOAT32 = 10,
    DFMI_TYPE_FLOAT64 = 11,
    DFMI_TYPE_UTF8 = 12
} dfmi_type;

/* Status codes: ExecutionError variants (error.rs:27-35) plus the ArrowError
 * kinds array_ops can raise, plus Rust panics and ABI failures. */
typedef enum dfmi_status {
    DFMI_OK = 0,
    DFMI_ERR_EXECUTION = 1,       /* ExecutionError::ExecutionError(String) */
    DFMI_ERR_GENERAL = 2,         /* ExecutionError::General(String) */
    DFMI_ERR_INVALID_COLUMN = 3,  /* ExecutionError::InvalidColumn(String) */
    DFMI_ERR_NOT_IMPLEMENTED = 4, /* ExecutionError::NotImplemented(String) */
    DFMI_ERR_DIVIDE_BY_ZERO = 5,  /* ExecutionError::ArrowError(DivideByZero) */
    DFMI_ERR_ARROW_COMPUTE = 6,   /* ExecutionError::ArrowError(ComputeError) */
    DFMI_ERR_PANIC = 7,           /* the reference panics (unwrap / i64 overflow) */
    DFMI_ERR_INVALID_ARGUMENT = 8,/* ABI misuse (bad pointer, alignment, sizes) */
    DFMI_ERR_CAPACITY = 9,        /* caller-provided output buffer too small */
    DFMI_ERR_DEVICE = 10,         /* HIP runtime failure / device timeout */
    DFMI_ERR_ARROW_PARSE = 11     /* ExecutionError::ArrowError(ParseError): CSV field */
} dfmi_status;

typedef struct dfmi_error {
    int32_t code;       /* dfmi_status */
    char message[500];  /* the reference's message text for that error */
} dfmi_error;

/* ---------------------------------------------------------------------------
 * Columnar batch (Arrow 0.12 memory layout, arrow::record_batch::RecordBatch).
 *   fixed width: `values` holds length * width bytes, native little-endian;
 *   Boolean: `values` is an LSB-first bitmap;
 *   Utf8 (BinaryArray): `offsets` holds length+1 int32, `values` the bytes.
 * `validity` is an LSB-first bitmap, NULL when the column has no nulls.
 * Bitmaps and values must be 8-byte aligned; device pointers for execution.
 * ------------------------------------------------------------------------- */
typedef struct dfmi_column {
    int32_t type;            /* dfmi_type */
    int32_t reserved;
    int64_t length;          /* rows */
    int64_t null_count;
    const uint8_t* validity; /* NULL => all valid */
    const void* values;
    const int32_t* offsets;  /* Utf8 only */
    /* arrow 0.12 ArrayData::offset (a sliced array): logical row i is physical
     * slot offset + i -- values[offset + i], validity / Boolean bit offset + i,
     * Utf8 offsets[offset + i] -- as value(i) / is_null(i) read it
     * (filter.rs:88-89,99-100). 0 for an unsliced array. */
    int64_t offset;
} dfmi_column;

typedef struct dfmi_batch {
    int32_t num_columns;
    int32_t reserved;
    int64_t num_rows;
    const dfmi_column* columns;
} dfmi_batch;

typedef struct dfmi_field {     /* arrow::datatypes::Field */
    const char* name;
    int32_t type;               /* dfmi_type */
    int32_t nullable;
} dfmi_field;

typedef struct dfmi_schema {    /* arrow::datatypes::Schema */
    int32_t num_fields;
    int32_t reserved;
    const dfmi_field* fields;
} dfmi_schema;

/* ---------------------------------------------------------------------------
 * Expressions: logicalplan::Expr (logicalplan.rs:133-164) flattened to
 * postfix order (children first, left before right), i.e. the order in which
 * compile_scalar_expr (expression.rs:244) evaluates them.
 * ------------------------------------------------------------------------- */
typedef enum dfmi_expr_kind {
    DFMI_EXPR_COLUMN = 1,             /* Expr::Column(index) */
    DFMI_EXPR_LITERAL = 2,            /* Expr::Literal(ScalarValue) */
    DFMI_EXPR_BINARY = 3,             /* Expr::BinaryExpr{left, op, right} */
    DFMI_EXPR_CAST = 4,               /* Expr::Cast{expr, data_type} */
    DFMI_EXPR_IS_NULL = 5,            /* Expr::IsNull */
    DFMI_EXPR_IS_NOT_NULL = 6,        /* Expr::IsNotNull */
    DFMI_EXPR_SORT = 7,               /* Expr::Sort */
    DFMI_EXPR_SCALAR_FUNCTION = 8,    /* Expr::ScalarFunction */
    DFMI_EXPR_AGGREGATE_FUNCTION = 9  /* Expr::AggregateFunction */
} dfmi_expr_kind;

typedef enum dfmi_operator {          /* logicalplan::Operator (logicalplan.rs:67-81) */
    DFMI_OP_EQ = 0,
    DFMI_OP_NOT_EQ = 1,
    DFMI_OP_LT = 2,
    DFMI_OP_LT_EQ = 3,
    DFMI_OP_GT = 4,
    DFMI_OP_GT_EQ = 5,
    DFMI_OP_PLUS = 6,
    DFMI_OP_MINUS = 7,
    DFMI_OP_MULTIPLY = 8,
    DFMI_OP_DIVIDE = 9,
    DFMI_OP_MODULUS = 10,
    DFMI_OP_AND = 11,
    DFMI_OP_OR = 12
} dfmi_operator;

typedef struct dfmi_expr_node {
    int32_t kind;       /* dfmi_expr_kind */
    int32_t op;         /* BINARY: dfmi_operator; SORT: asc (1/0) */
    int32_t data_type;  /* LITERAL: ScalarValue variant; CAST/functions: target type */
    int32_t column;     /* COLUMN: index; functions: argument count */
    int64_t i64;        /* LITERAL Int*, UInt* (bit pattern), Boolean (0/1) */
    double f64;         /* LITERAL Float32/Float64 (Float32 stored widened) */
    const char* str;    /* LITERAL Utf8 bytes; functions: name */
    int64_t str_len;
} dfmi_expr_node;

/* Extension flags. 0 = exactly the reference's behaviour. */
#define DFMI_FLAG_EXT_GATHER_ALL   0x1u /* filter Int64 (and other fixed-width) columns
                                           instead of "filter not supported for ..." */
#define DFMI_FLAG_EXT_UTF8_COMPARE 0x2u /* Utf8 literals and Utf8 =/!= comparisons
                                           instead of "No support for literal type" */
#define DFMI_FLAG_EXT_CAST         0x4u /* CAST(<numeric expression> AS <numeric type>)
                                           instead of "column reference" / "CAST not
                                           implemented for expression" (expression.rs:281-290,
                                           321-324): arrow 0.12 cast kernel rules -- a null
                                           stays null, a value the target type cannot hold
                                           (num::cast -> None: out of range, NaN to an
                                           integer) becomes null. Literal casts stay exactly
                                           the reference's (Int64 -> Float64 only). */
#define DFMI_FLAG_EXT_IS_NULL      0x8u /* IsNull / IsNotNull (expression.rs:326-345,
                                           commented out in the reference): the operand's
                                           validity as a non-null Boolean */

#define DFMI_FLAG_EXT_AGGREGATE    0x10u /* LogicalPlan::Aggregate, with or without GROUP BY
                                           (sqlplanner.rs:91-117, compile_expr
                                           expression.rs:81-116) instead of the
                                           executor's unimplemented!() (context.rs:161):
                                           MIN / MAX / SUM / COUNT over the selected
                                           rows, semantics in DESIGN.md §2 */

/* Opaque compiled expression: the RuntimeExpr::Compiled of expression.rs:43-50. */
typedef struct dfmi_program dfmi_program;

/* compile_scalar_expr (expression.rs:244-451). Rejects exactly what the
 * reference rejects at compile time, with the same error variant and text.
 * Errors the reference raises only when the closure runs (comparison_ops,
 * math_ops, panics) are recorded in the program and reported by execution. */
int32_t dfmi_compile_scalar_expr(const dfmi_expr_node* nodes, int32_t num_nodes,
                                 const dfmi_schema* input_schema, uint32_t flags,
                                 dfmi_program** out, dfmi_error* err);

/* RuntimeExpr::get_name / get_type (expression.rs:64-77). */
const char* dfmi_program_name(const dfmi_program* program);
int32_t dfmi_program_type(const dfmi_program* program);
void dfmi_program_free(dfmi_program* program);

/* ---------------------------------------------------------------------------
 * Execution context: one per (GPU, stream). Holds the look-back tile-status
 * workspace, result counters and error words. Not thread-safe; one host
 * thread per context (the reference is single-threaded, context.rs:33).
 * ------------------------------------------------------------------------- */
typedef struct dfmi_context dfmi_context;

int32_t dfmi_context_create(int32_t device, void* hip_stream, dfmi_context** out,
                            dfmi_error* err);
void dfmi_context_destroy(dfmi_context* ctx);
/* Rebind the stream used by later calls (e.g. torch's current stream). */
int32_t dfmi_context_set_stream(dfmi_context* ctx, void* hip_stream);

/* Output column. The caller provides device buffers sized for the worst case:
 *   values:   num_rows * width bytes (Boolean: ceil(num_rows/8), 8-padded);
 *   validity: ceil(num_rows/8) bytes, 8-padded; written when the result can
 *             hold nulls (always without a predicate; after a Selection only
 *             for a projection with a fallible CAST, DFMI_FLAG_EXT_CAST) --
 *             null_count > 0 says it holds the result's validity;
 *   offsets:  (num_rows+1) int32 for Utf8;
 *   data:     Utf8 bytes, data_capacity >= input column's byte length.
 * The library fills the fields below the line. */
typedef struct dfmi_out_column {
    void* values;
    uint8_t* validity;
    int32_t* offsets;
    uint8_t* data;
    int64_t data_capacity;
    /* ---- filled by dfmi_filter_project ---- */
    int32_t type;                /* dfmi_type of the result array */
    int32_t passthrough_column;  /* >=0: result IS that input column (Arc clone,
                                    expression.rs:272-276); buffers untouched */
    int64_t length;
    int64_t null_count;          /* 0 => validity not written / not needed */
    int64_t data_length;         /* Utf8 bytes written */
} dfmi_out_column;

/* One pull of ProjectRelation::next(FilterRelation::next(batch))
 * (projection.rs:45-66, filter.rs:46-72, filter() filter.rs:80-111),
 * fused into one pass over HBM.
 *   predicate == NULL       : no Selection in the plan (projection only);
 *   num_projections == 0    : no Projection: FilterRelation output = every
 *                             input column filtered (outputs has num_columns);
 * The call is synchronous: on return `outputs[i].length` is the batch's row
 * count. Errors are the ones the reference's next() returns. */
int32_t dfmi_filter_project(dfmi_context* ctx, const dfmi_program* predicate,
                            const dfmi_program* const* projections, int32_t num_projections,
                            const dfmi_batch* input, dfmi_out_column* outputs,
                            uint32_t flags, dfmi_error* err);

/* ---------------------------------------------------------------------------
 * Coalesced form for small batches: the pull of dfmi_filter_project on each
 * of `num_batches` device batches IN ORDER, as the reference's pull loop
 * runs them one next() at a time (csv_sql.rs:49 reads 1024-row batches and
 * pulls them in csv_sql.rs:60-62; relation.rs:27-32), but as ONE kernel
 * launch for all of them. Batches share the schema (column types); each has
 * its own rows, buffers and outputs: `outputs` holds num_batches x n
 * columns, batch-major (n = num_projections, or num_columns without a
 * projection), each sized for its own batch as in dfmi_filter_project. Every
 * batch gets exactly the output dfmi_filter_project would give it (one
 * output batch per input batch, 0-row batches included).
 * Errors: the call returns the error of the first batch that raises one;
 * *failed_batch names it and the batches before it are complete -- the
 * caller hands those out first, as the pull loop would have seen them. A
 * plan error the reference raises on every batch fails batch 0.
 * ------------------------------------------------------------------------- */
int32_t dfmi_filter_project_batches(dfmi_context* ctx, const dfmi_program* predicate,
                                    const dfmi_program* const* projections, int32_t num_projections,
                                    const dfmi_batch* inputs, int32_t num_batches, dfmi_out_column* outputs,
                                    uint32_t flags, int32_t* failed_batch, dfmi_error* err);

/* ---------------------------------------------------------------------------
 * Host-buffer form, for callers whose batches live in host memory (the Rust
 * reference's arrow 0.12 buffers from csv::Reader, csv_sql.rs:49): the same
 * pull as dfmi_filter_project -- FilterRelation::next (filter.rs:46-72) +
 * filter() (filter.rs:80-111) + ProjectRelation::next (projection.rs:45-66)
 * -- but `input` holds HOST pointers. Rows are independent, so the library
 * cuts the batch into row chunks (~48 MiB of input each) and pipelines them:
 * host staging copies, H2D DMA, the fused pass and D2H DMA of consecutive
 * chunks overlap; chunk results are concatenated in row order into host
 * buffers the library owns until dfmi_host_result_free. The result and any
 * error are those of one pull over the whole batch (the first error in the
 * reference's evaluation order over all rows). Passthrough columns (Arc
 * clones, expression.rs:272-276) are returned as copies.
 * ------------------------------------------------------------------------- */
typedef struct dfmi_host_result dfmi_host_result;

int32_t dfmi_filter_project_host(dfmi_context* ctx, const dfmi_program* predicate,
                                 const dfmi_program* const* projections, int32_t num_projections,
                                 const dfmi_batch* input, uint32_t flags,
                                 dfmi_host_result** out, dfmi_error* err);
int32_t dfmi_host_result_num_columns(const dfmi_host_result* result);
/* Host view of result column i; buffers stay valid until the result is freed.
 * `validity` is NULL when null_count == 0 (filtered outputs never have one). */
int32_t dfmi_host_result_column(const dfmi_host_result* result, int32_t i, dfmi_column* view);
/* Views of columns [first, first + count) in one call (views[k] as
 * dfmi_host_result_column(first + k)): a binding that hands out one output
 * batch per input batch of the coalesced form below reads every batch's
 * views at once instead of one FFI call per column. */
int32_t dfmi_host_result_columns(const dfmi_host_result* result, int32_t first, int32_t count, dfmi_column* views);
/* The one pinned block holding the columns of a coalesced result (NULL / 0
 * for the single-batch pipelined form): a binding may wrap it once and slice
 * every column's buffers out of it, keeping the result alive while any such
 * slice is. Passthrough columns live outside it. */
int32_t dfmi_host_result_block(const dfmi_host_result* result, const void** base, size_t* bytes);
void dfmi_host_result_free(dfmi_host_result* result);

/* Coalesced form of dfmi_filter_project_host for many small HOST batches
 * (csv_sql.rs:49-62: 1024-row batches read from csv::Reader, pulled one
 * next() at a time): the batches' buffers are packed into pinned memory, moved
 * with one H2D copy, run as one dfmi_filter_project_batches launch, and the
 * outputs come back with one D2H copy. The result holds num_batches x n
 * columns, batch-major (n = num_projections, or num_columns without a
 * projection). Errors as dfmi_filter_project_batches: the call returns the
 * error of the first batch that raises one and *failed_batch names it; the
 * result is still returned, with the batches before it complete and the rest
 * empty (the caller hands those out first). Free the result in every case. */
int32_t dfmi_filter_project_host_batches(dfmi_context* ctx, const dfmi_program* predicate,
                                         const dfmi_program* const* projections, int32_t num_projections,
                                         const dfmi_batch* inputs, int32_t num_batches, uint32_t flags,
                                         dfmi_host_result** out, int32_t* failed_batch, dfmi_error* err);

/* Caller-owned form of dfmi_filter_project_host_batches: the outputs are
 * written into ONE host block the caller allocated (e.g. an arrow 0.12
 * MutableBuffer, which freezes into the Buffer every output array slices --
 * projection.rs:59-60 / filter.rs:60-61 return freshly built arrays per pull),
 * instead of a library-owned result. dfmi_host_batches_output_bytes gives the
 * block's worst-case size for these batches (every row selected); the block
 * must be 64-byte aligned. Each output buffer starts at a 256-byte multiple
 * of the block. `outputs` (num_batches x n, batch-major, n = num_projections
 * or num_columns without a projection) is filled by the library: values /
 * validity (null_count > 0) / Utf8 offsets + data point into the block;
 * passthrough_column >= 0 marks an output that IS that input column (the Arc
 * clone of expression.rs:272-276: the caller reuses its own input array).
 * A block in pinned memory (dfmi_host_alloc, dfmi_host_register, any
 * hipHostMalloc'd allocation) is written by the kernel in place; a pageable
 * block receives the selected bytes with one host copy from the library's
 * pinned staging. Errors and *failed_batch as dfmi_filter_project_host_batches
 * (the batches before the failing one are complete);
 * out_capacity < the size needed -> DFMI_ERR_CAPACITY, nothing run. */
int32_t dfmi_host_batches_output_bytes(const dfmi_program* predicate, const dfmi_program* const* projections,
                                       int32_t num_projections, const dfmi_batch* inputs, int32_t num_batches,
                                       uint32_t flags, size_t* bytes, dfmi_error* err);
int32_t dfmi_filter_project_host_batches_into(dfmi_context* ctx, const dfmi_program* predicate,
                                              const dfmi_program* const* projections, int32_t num_projections,
                                              const dfmi_batch* inputs, int32_t num_batches, uint32_t flags,
                                              void* out_block, size_t out_capacity, dfmi_out_column* outputs,
                                              int32_t* failed_batch, dfmi_error* err);

/* Pinned host memory for batch buffers (e.g. a CSV reader parsing straight
 * into them; csv_sql.rs:49's DataSource side). Columns whose buffers lie in
 * such memory -- or in any hipHostMalloc'd allocation of at least 1 MiB --
 * are DMA'd by dfmi_filter_project_host straight from the caller's memory
 * instead of through the library's pinned staging. dfmi_host_register pins
 * an existing range (hipHostRegister) until dfmi_host_unregister. */
int32_t dfmi_host_alloc(size_t bytes, void** out, dfmi_error* err);
int32_t dfmi_host_free(void* ptr);
int32_t dfmi_host_register(void* ptr, size_t bytes, dfmi_error* err);
int32_t dfmi_host_unregister(void* ptr);

/* The context's GPU is shared with other processes (several ranks on one
 * device, a time-sliced GPU): kernels with a decoupled look-back take their
 * tiles from an atomic ticket counter from the first launch, so a tile never
 * waits on a predecessor another process keeps off the CUs.
 * Default: off, or DFMI_SHARED=1 in the environment at dfmi_context_create.
 * Without it a shared launch still completes, after a 2 s look-back timeout
 * and a ticket-ordered relaunch. */
int32_t dfmi_context_set_shared(dfmi_context* ctx, int32_t shared);

/* HIP events around each launch (default on): dfmi_last_timing needs them;
 * off saves two event records per call on the small-batch path. */
int32_t dfmi_context_set_timing(dfmi_context* ctx, int32_t enable);

/* Device time in milliseconds of the last dfmi_filter_project's kernels
 * (HIP events on the context stream), and the dominant kernel's share. */
int32_t dfmi_last_timing(const dfmi_context* ctx, double* total_ms, double* main_kernel_ms);

/* hipRTC compile time in milliseconds of the last dfmi_filter_project call
 * (0 when its query shape was already compiled: the kernel cache is keyed by
 * the programs and the batch's column types / nullability). */
int32_t dfmi_last_compile_ms(const dfmi_context* ctx, double* compile_ms);

/* Name of the query kernel the last dfmi_filter_project / dfmi_aggregate_batch
 * on ctx launched: dfmi_<filter|project|agg>_<hash of the generated code>, as
 * rocprofv3 reports it ("" before the first launch). Diagnostics. */
const char* dfmi_last_kernel_name(const dfmi_context* ctx);

/* Evaluation-order key of the error the last dfmi_filter_project on ctx
 * returned: (position of the failing operator in the reference's evaluation
 * order) << 44 | row << 4; all ones when it returned no such error. Lets a
 * sharded caller report the error the reference would raise first over the
 * whole table (smallest key position, then the earliest shard). */
int32_t dfmi_last_error_order(const dfmi_context* ctx, uint64_t* key);

/* ---------------------------------------------------------------------------
 * Aggregate extension (DFMI_FLAG_EXT_AGGREGATE). The reference plans
 * `SELECT SUM(e), ... FROM t [WHERE p]` as Aggregate(Selection?(TableScan))
 * (sqlplanner.rs:91-117) and compiles each AggregateFunction with
 * compile_expr (expression.rs:81-116: one argument compiled by
 * compile_scalar_expr, AggregateType Min/Max/Count/Sum), but its executor
 * stops at `unimplemented!()` (context.rs:161). Here the whole pull --
 * FilterRelation::next over every batch plus the aggregation -- is one fused
 * pass per batch (no filtered batch is materialised), accumulated in a
 * device state across batches. Semantics (build-defined, oracle-pinned):
 *   COUNT(e): non-null values of e over the selected rows (UInt64);
 *   SUM(e):   integers wrap in e's type; Float32/Float64 are the exact sum
 *             rounded once (round half to even) -- independent of order,
 *             batch and GPU count; a NaN input or +inf with -inf gives the
 *             canonical quiet NaN, otherwise an infinite input gives that
 *             infinity; an exact zero is -0.0 only if every value is -0.0;
 *   MIN/MAX(e): NaN values are skipped (a set of only NaNs gives the
 *             canonical NaN), -0.0 orders below +0.0;
 *   SUM/MIN/MAX over no non-null value is null.
 * GROUP BY (dfmi_agg_state_create_grouped / _multi): one to four key
 * expressions of any type the reference's values take -- Boolean, integer,
 * Float32 / Float64 or Utf8; per group the aggregates above. Groups come out
 * in key order, lexicographic over the key parts, each part ordered false <
 * true, integers numerically, floats by IEEE 754 totalOrder with one group per
 * bit pattern -- -NaN < -inf < ... < -0.0 < +0.0 < ... < +inf < +NaN, as
 * Rust's total_cmp --, Utf8 bytewise, with that part's null last -- for one
 * Boolean key the order of the reference's expected/csv_aggregate_by_c_bool.csv.
 * One Boolean / integer key: a batch whose selected keys lie within 16
 * consecutive values runs the fused grouped kernel. Every other batch (wider
 * integer keys, float or Utf8 keys, several keys) runs the keys and the
 * arguments through the fused Selection + Projection pass, then a device hash
 * table (open addressing, one claim pass and one accumulate pass with the
 * same per-row rules; rows whose key shares its 63-bit hash with another
 * key's are merged on the host) -- any number of groups per batch and
 * overall (up to 2^30 per device).
 * ------------------------------------------------------------------------- */
typedef enum dfmi_agg_fn {       /* AggregateType (expression.rs:33-40) */
    DFMI_AGG_MIN = 0,
    DFMI_AGG_MAX = 1,
    DFMI_AGG_SUM = 2,
    DFMI_AGG_COUNT = 3
} dfmi_agg_fn;

typedef struct dfmi_agg_value {
    int32_t type;      /* dfmi_type of the result (the AggregateFunction return_type) */
    int32_t is_null;   /* 1: no non-null input value (SUM / MIN / MAX) */
    int64_t count;     /* non-null input values aggregated */
    uint64_t bits;     /* integers sign/zero-extended to 64 bits, Float32 bits in the
                          low 32, Float64 bits */
} dfmi_agg_value;

typedef struct dfmi_aggregate dfmi_aggregate;

/* compile_expr's AggregateFunction arm (expression.rs:81-116): `name` as the
 * SQL text spells it (min / max / sum / count, any case; anything else panics
 * in the reference: DFMI_ERR_PANIC), `argument` compiled by
 * dfmi_compile_scalar_expr, `return_type` the planner's (sqlplanner.rs:296-330:
 * the argument's type, UInt64 for count). */
int32_t dfmi_compile_aggregate(const char* name, const dfmi_program* argument, int32_t return_type,
                               uint32_t flags, dfmi_aggregate** out, dfmi_error* err);
const char* dfmi_aggregate_name(const dfmi_aggregate* agg);
int32_t dfmi_aggregate_type(const dfmi_aggregate* agg);
void dfmi_aggregate_free(dfmi_aggregate* agg);

/* Device accumulators of one Aggregate plan on one context. */
typedef struct dfmi_agg_state dfmi_agg_state;

int32_t dfmi_agg_state_create(dfmi_context* ctx, const dfmi_aggregate* const* aggs, int32_t num_aggs,
                              dfmi_agg_state** out, dfmi_error* err);
/* One batch of the aggregate's input (FilterRelation::next when predicate is
 * non-NULL), accumulated on the device; asynchronous on the context stream
 * except for error reporting, which is synchronous like dfmi_filter_project. */
int32_t dfmi_aggregate_batch(dfmi_context* ctx, dfmi_agg_state* state, const dfmi_program* predicate,
                             const dfmi_batch* input, uint32_t flags, dfmi_error* err);
/* The aggregate values over every batch so far (num_aggs entries). */
int32_t dfmi_agg_state_finish(dfmi_context* ctx, dfmi_agg_state* state, dfmi_agg_value* out,
                              dfmi_error* err);
/* Multi-GPU: the exact partial state (count, flags, min/max key, integer sum,
 * exact float sum digits) as dfmi_agg_partial_bytes() host bytes, and the
 * merge of partials from every shard into final values -- bit-identical to
 * one state over all the shards' rows. */
int64_t dfmi_agg_partial_bytes(const dfmi_agg_state* state);
int32_t dfmi_agg_state_partial(dfmi_context* ctx, dfmi_agg_state* state, void* host_out, dfmi_error* err);
int32_t dfmi_agg_merge_partials(const dfmi_aggregate* const* aggs, int32_t num_aggs,
                                const void* const* partials, int32_t num_partials, dfmi_agg_value* out,
                                dfmi_error* err);
/* GROUP BY extension: LogicalPlan::Aggregate{group_expr: [key]}
 * (sqlplanner.rs:91-117; the reference's executor stops at context.rs:161).
 * `key` compiled by dfmi_compile_scalar_expr over the same schema (Boolean,
 * integer, Float32 / Float64 or Utf8), at most 15 aggregates. Batches go
 * through dfmi_aggregate_batch. */
int32_t dfmi_agg_state_create_grouped(dfmi_context* ctx, const dfmi_program* key, const dfmi_aggregate* const* aggs,
                                      int32_t num_aggs, dfmi_agg_state** out, dfmi_error* err);
/* ... with group_expr = keys[0..num_keys) (1 to 4 expressions, the
 * planner's Vec<Expr>, sqlplanner.rs:97-103), evaluated in that order before
 * the aggregates' arguments (their errors come first, in that order). */
int32_t dfmi_agg_state_create_grouped_multi(dfmi_context* ctx, const dfmi_program* const* keys, int32_t num_keys,
                                            const dfmi_aggregate* const* aggs, int32_t num_aggs, dfmi_agg_state** out,
                                            dfmi_error* err);
/* The state's GROUP BY expressions (0: not a grouped state). */
int32_t dfmi_agg_state_num_keys(const dfmi_agg_state* state);
/* The groups so far, in key order: keys[g * num_keys + p] for key part p
 * (type = the part's type, is_null, bits: Boolean 0/1, integers
 * sign/zero-extended, float bits, Utf8 0 -- the bytes come from
 * dfmi_agg_state_group_keys_utf8_part; count = the group's selected rows) and
 * values[g * num_aggs + j]. *num_groups is set even when it exceeds
 * `capacity` (groups; then DFMI_ERR_INVALID_ARGUMENT and nothing is
 * written). */
int32_t dfmi_agg_state_finish_grouped(dfmi_context* ctx, dfmi_agg_state* state, int64_t capacity, dfmi_agg_value* keys,
                                      dfmi_agg_value* values, int64_t* num_groups, dfmi_error* err);
/* The Utf8 key part `part` of the groups of the last
 * dfmi_agg_state_finish_grouped (or dfmi_shard_agg_finish_grouped), in the
 * same order, as an arrow BinaryArray: offsets[0..num_groups] (from 0) and
 * the bytes (a null key's slot is empty; keys[g * num_keys + part].is_null
 * says which). *data_length is set even when a capacity is too small (then
 * DFMI_ERR_CAPACITY and nothing is written). _utf8: part 0. */
int32_t dfmi_agg_state_group_keys_utf8_part(const dfmi_agg_state* state, int32_t part, int32_t* offsets,
                                            int64_t num_offsets, uint8_t* data, int64_t data_capacity,
                                            int64_t* data_length, dfmi_error* err);
int32_t dfmi_agg_state_group_keys_utf8(const dfmi_agg_state* state, int32_t* offsets, int64_t num_offsets, uint8_t* data,
                                       int64_t data_capacity, int64_t* data_length, dfmi_error* err);
/* Multi-GPU GROUP BY: the exact per-group partial state (every key part --
 * Utf8 bytes included --, the group's selected rows, every aggregate's
 * partial) as host bytes -- size first (negative: -status) -- and the merge
 * of every shard's bytes into the groups one state over all the shards' rows
 * would hold, in key order (output as dfmi_agg_state_finish_grouped; the
 * bytes of a Utf8 key part of the merged groups from
 * dfmi_agg_merge_grouped_partials_keys_utf8, same order). */
int64_t dfmi_agg_state_grouped_partial_bytes(dfmi_context* ctx, dfmi_agg_state* state, dfmi_error* err);
int32_t dfmi_agg_state_grouped_partial(dfmi_context* ctx, dfmi_agg_state* state, void* host_out, int64_t bytes,
                                       dfmi_error* err);
int32_t dfmi_agg_merge_grouped_partials(const dfmi_aggregate* const* aggs, int32_t num_aggs,
                                        const void* const* partials, const int64_t* sizes, int32_t num_partials,
                                        int64_t capacity, dfmi_agg_value* keys, dfmi_agg_value* values,
                                        int64_t* num_groups, dfmi_error* err);
int32_t dfmi_agg_merge_grouped_partials_keys_utf8(const dfmi_aggregate* const* aggs, int32_t num_aggs,
                                                  const void* const* partials, const int64_t* sizes,
                                                  int32_t num_partials, int32_t part, int32_t* offsets,
                                                  int64_t num_offsets, uint8_t* data, int64_t data_capacity,
                                                  int64_t* data_length, dfmi_error* err);
/* Back to the empty state (asynchronous on the context stream): re-running the query. */
int32_t dfmi_agg_state_reset(dfmi_context* ctx, dfmi_agg_state* state, dfmi_error* err);
void dfmi_agg_state_free(dfmi_agg_state* state);

/* ---------------------------------------------------------------------------
 * Multi-GPU. The reference is single-threaded (context.rs:33);
 * its pull is Relation::next (relation.rs:27-32). Rows are independent
 * through the Selection / Projection path and filter() keeps row order
 * (filter.rs:87-91), so a table shards by row range: one host thread or
 * process per GPU, each with its own context, calls the shard entry points
 * below on its own rows; per-rank outputs in rank order are the reference's
 * output stream. The only collective is one RCCL all_gather of a few int64
 * per rank after each pass (placement and errors); gathering results on one
 * rank is optional (grouped send/recv over xGMI).
 * ------------------------------------------------------------------------- */
#define DFMI_SHARD_ID_BYTES 128
typedef struct dfmi_shard_comm dfmi_shard_comm;

typedef struct dfmi_shard_placement {
    int32_t world, rank;
    int64_t row_offset;       /* first global output row of this rank's outputs */
    int64_t total_rows;       /* output rows over all ranks */
    int64_t utf8_base[16];    /* per output: global byte offset of this rank's Utf8 data */
    int64_t utf8_total[16];   /* per output: Utf8 bytes over all ranks */
    int64_t null_total[16];   /* per output: nulls over all ranks */
} dfmi_shard_placement;

/* A new RCCL unique id (rank 0), to be handed to every rank out of band. */
int32_t dfmi_shard_unique_id(uint8_t* id /* DFMI_SHARD_ID_BYTES */, dfmi_error* err);
/* Collective over `world` ranks (ncclCommInitRank on the context's device). */
int32_t dfmi_shard_comm_init(dfmi_context* ctx, int32_t world, int32_t rank, const uint8_t* id,
                             dfmi_shard_comm** out, dfmi_error* err);
void dfmi_shard_comm_destroy(dfmi_shard_comm* comm);
/* dfmi_filter_project over this rank's rows, then the placement exchange.
 * Collective: every rank calls it. When any rank fails, every rank returns
 * the error the reference would raise over the whole table (the smallest
 * evaluation position, then the earliest rows). */
int32_t dfmi_shard_filter_project(dfmi_context* ctx, dfmi_shard_comm* comm, const dfmi_program* predicate,
                                  const dfmi_program* const* projections, int32_t num_projections,
                                  const dfmi_batch* input, dfmi_out_column* outputs, uint32_t flags,
                                  dfmi_shard_placement* placement, dfmi_error* err);
/* Concatenate the last dfmi_shard_filter_project outputs on `root`, in rank
 * order (collective). `root_outputs` (root only) are device buffers sized for
 * placement.total_rows / utf8_total; Utf8 offsets are rebased, bitmaps
 * re-aligned. Fails (Capacity) if a gathered Utf8 column would pass 2^31 bytes. */
int32_t dfmi_shard_gather_to_root(dfmi_context* ctx, dfmi_shard_comm* comm, const dfmi_out_column* local_outputs,
                                  const dfmi_out_column* root_outputs, int32_t root, dfmi_error* err);
/* Aggregate extension across ranks (collective): every rank's exact partial
 * all_gathered and merged -- the values one GPU would produce over all rows. */
int32_t dfmi_shard_agg_finish(dfmi_context* ctx, dfmi_shard_comm* comm, dfmi_agg_state* state,
                              const dfmi_aggregate* const* aggs, int32_t num_aggs, dfmi_agg_value* out,
                              dfmi_error* err);
/* ... with a GROUP BY key (collective): every rank's per-group partials
 * all_gathered and merged; output as dfmi_agg_state_finish_grouped (every
 * rank gets the same groups; *num_groups set even past `capacity`). */
int32_t dfmi_shard_agg_finish_grouped(dfmi_context* ctx, dfmi_shard_comm* comm, dfmi_agg_state* state,
                                      const dfmi_aggregate* const* aggs, int32_t num_aggs, int64_t capacity,
                                      dfmi_agg_value* keys, dfmi_agg_value* values, int64_t* num_groups,
                                      dfmi_error* err);

#ifdef __cplusplus
}
#endif
#endif /* DFMI_H */
