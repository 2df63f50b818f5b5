// Host-side compiled expression (the RuntimeExpr of expression.rs:43-50).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/dfmi.h"

namespace dfmi {

// IR_CAST (DFMI_FLAG_EXT_CAST): child l converted to `type` with the arrow
// cast kernel's rules; IR_ISNULL (DFMI_FLAG_EXT_IS_NULL): op 0 = IS NULL,
// 1 = IS NOT NULL of child l.
enum IrKind { IR_COL = 1, IR_LIT = 2, IR_BIN = 3, IR_CAST = 4, IR_ISNULL = 5 };

struct IrNode {
    int kind = 0;
    int type = 0;        // result dfmi_type
    int op = 0;          // IR_BIN: dfmi_operator; IR_ISNULL: 0 / 1
    int col = -1;        // IR_COL
    int l = -1, r = -1;  // IR_BIN children, IR_CAST / IR_ISNULL child (IR indices)
    uint64_t bits = 0;   // IR_LIT numeric payload (raw 64-bit, Float32 widened bits)
    std::string str;     // IR_LIT Utf8 payload
    std::string name;    // RuntimeExpr name of this sub-expression
    int ordinal = 0;     // postfix position = evaluation order
    // Error the closure raises when it runs (comparison_ops / math_ops /
    // boolean_ops unwrap panic); 0 = none.
    int32_t rt_code = 0;
    std::string rt_msg;
};

const char* type_debug(int t);
bool is_numeric_type(int t);
std::string rust_float(double v, bool f32, bool debug);

}  // namespace dfmi

struct dfmi_program {
    uint64_t uid = 0;               // unique per compiled program (never reused): kernel cache key
    std::string name;
    int type = 0;
    uint32_t flags = 0;
    int length = 0;                 // postfix node count (ordinal space)
    std::vector<int> schema_types;  // input schema it was compiled against
    std::vector<dfmi::IrNode> ir;   // postfix order
    int root = -1;
};
