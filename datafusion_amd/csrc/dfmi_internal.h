// Internal device-program format of libdfmi (not part of the C ABI).
//
// A compiled predicate / projection is lowered into an accumulator program:
//   numeric input columns   read-only register vector c[k][0..NC) per row k
//                           (dynamic reads lower to s_set_gpr_idx + v_mov);
//   accumulator             acc[k]: every math op writes it (static register);
//   temporaries             LDS s_tmp[t][row] for non-left-deep trees (SAVE);
//   boolean values          bits of bv[k] (validity bits of bvd[k]);
//   literals                kernarg (SGPR), never materialised per row.
// k = 0..K-1 indexes the K rows one thread owns inside a tile; K*NC = 16.
// Every instruction field is wave-uniform (kernarg -> SGPR): dispatch is a
// scalar branch. No dynamic register *writes*: those make the register
// allocator copy the whole vector per write (measured, DESIGN.md "Kernels").
#pragma once
#include <stdint.h>

namespace dfmi {

constexpr int kMaxNum = 16;     // numeric input columns per launch (NC <= 16)
constexpr int kMaxBoolCols = 8; // Boolean input columns per launch
constexpr int kMaxUtf8 = 4;     // Utf8 input columns per launch
constexpr int kMaxIns = 96;     // device instructions per launch
constexpr int kMaxLits = 24;    // 64-bit literals per launch
constexpr int kMaxStrLits = 4;
constexpr int kStrLitBytes = 128;
constexpr int kMaxOut = 16;     // output columns per launch
constexpr int kMaxTmp = 4;      // LDS temporaries
constexpr int kMaxChan = 1 + kMaxUtf8;  // look-back channels: rows + Utf8 bytes

enum DOp : uint8_t {
    OP_NOP = 0,
    // comparisons: bool slot dst <- cmp(operand a, operand b)
    OP_EQ_I64, OP_NE_I64, OP_LT_I64, OP_LE_I64, OP_GT_I64, OP_GE_I64,
    OP_EQ_F64, OP_NE_F64, OP_LT_F64, OP_LE_F64, OP_GT_F64, OP_GE_F64,
    // math: acc <- operand a OP operand b
    OP_ADD_I64, OP_SUB_I64, OP_MUL_I64, OP_DIV_I64,
    OP_ADD_F64, OP_SUB_F64, OP_MUL_F64, OP_DIV_F64,
    // boolean: bool slot dst <- bool slot a AND/OR bool slot b
    OP_AND, OP_OR,
    // Utf8 (extension): a = utf8 input index, b = string literal / utf8 index
    OP_EQ_UTF8_LIT, OP_NE_UTF8_LIT, OP_EQ_UTF8_COL, OP_NE_UTF8_COL,
    OP_SAVE,   // tmp[dst] <- acc
    OP_MOVE,   // acc <- operand a
    OP_BLIT,   // bool slot dst <- (b & 1)
    // output stores (dst = output index); compacted rows in k_filter_project,
    // dense rows + ballot-packed bitmaps in k_project
    OP_STORE_ACC,   // out[dst] <- acc
    OP_STORE_COL,   // out[dst] <- numeric column a (raw slot bits)
    OP_STORE_BOOL,  // out[dst] <- bool slot a
    OP_COUNT_
};

// operand kinds (DIns.ka / DIns.kb)
enum DKind : uint8_t { KD_COL = 0, KD_LIT = 1, KD_ACC = 2, KD_TMP = 3 };

struct DIns {
    uint8_t op;
    uint8_t dst;
    uint8_t a;
    uint8_t b;
    uint8_t ka;
    uint8_t kb;
    uint16_t ordinal;  // evaluation position (error ordering across exprs)
};

struct DCol {
    const void* values;       // numeric values / Boolean bits / Utf8 bytes
    const uint8_t* validity;  // nullptr => all valid
    const int32_t* offsets;   // Utf8 only
    int64_t bitmap_bytes;     // bytes readable at validity / Boolean values
};

enum DOutKind : int32_t {
    OUT_GATHER_NUM = 1,  // copy raw 8-byte column (filter.rs:84-93)
    OUT_EXPR_NUM = 2,    // run ins[begin,end), store acc
    OUT_EXPR_BOOL = 3,   // run ins[begin,end), store bool slot
    OUT_GATHER_UTF8 = 4, // Utf8 offset/byte gather (filter.rs:94-105)
    OUT_GATHER_BOOL = 5, // ext: Boolean column gather (bool slot)
};

struct DOut {
    int32_t kind;
    int32_t slot;        // utf8 input index (OUT_GATHER_UTF8)
    int32_t chan;        // look-back channel (Utf8 bytes)
    int32_t pad;
    int64_t data_cap;    // Utf8 output byte capacity
    void* values;        // numeric values; bool: temp bytes (filtered) or bits
    uint8_t* validity;   // projection-only kernel
    int32_t* offsets;    // Utf8
    uint8_t* data;       // Utf8 bytes
};

// Everything a launch needs, passed by value as the kernel argument.
struct DLaunch {
    int64_t n_rows;
    int32_t n_tiles;
    int32_t n_num;
    int32_t n_bool;
    int32_t n_utf8;
    int32_t pred_begin;
    int32_t pred_end;
    int32_t pred_slot;
    int32_t proj_begin;
    int32_t proj_end;
    int32_t n_out;
    int32_t n_chan;
    int32_t n_tmp;
    int32_t chan_out[kMaxUtf8];   // Utf8 byte channel 1+u -> output index
    int32_t mode;                 // diagnostics: bit0 tile=blockIdx, bit1 no look-back
    int32_t n_lds;                // numeric columns 0..n_lds-1 staged in LDS
    DCol num[kMaxNum];
    DCol boolc[kMaxBoolCols];
    DCol utf8[kMaxUtf8];
    DIns ins[kMaxIns];
    uint64_t lits[kMaxLits];
    int32_t strlit_off[kMaxStrLits];
    int32_t strlit_len[kMaxStrLits];
    char strlit[kStrLitBytes];
    DOut out[kMaxOut];
    unsigned long long* status;   // [n_chan][n_tiles] look-back words
    unsigned int* ticket;         // dynamic tile ticket
    unsigned long long* err;      // max(~key) error word, 0 = none
    unsigned long long* totals;   // [kMaxChan] rows / bytes; [kMaxChan..] null counts
};

// error word: key = ordinal << 44 | row << 4 | kind; stored inverted so
// atomicMax keeps the smallest key (the reference's first failing row of the
// first failing operator).
enum DErrKind : uint32_t {
    ERRK_DIV_ZERO = 1,
    ERRK_DIV_OVERFLOW = 2,
    ERRK_LOOKBACK_TIMEOUT = 3,
    ERRK_CAPACITY = 4,
};

}  // namespace dfmi
