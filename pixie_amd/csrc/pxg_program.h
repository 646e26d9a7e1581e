// Host-side validation of pxg_program and lowering to the device representation.
#pragma once

#include <vector>

#include "pxg_internal.h"

namespace pxg {

inline bool IsFixedBinOp(int op) {
  return (op >= PXG_OP_ADD_I && op <= PXG_OP_BIN_I) || (op >= PXG_OP_ADD_F && op <= PXG_OP_DIV_F) ||
         (op >= PXG_OP_EQ_I && op <= PXG_OP_GE_I) || (op >= PXG_OP_EQ_F && op <= PXG_OP_APPROX_NE_F) || op == PXG_OP_AND ||
         op == PXG_OP_OR;
}

// Type-checks `in` against the input column types, lowers it into `out`.  The constant pool
// is appended to `pool` (the caller uploads it and patches DevProgram::pool with
// SetPoolBase).  `pool_off` receives the offset of this program's pool in `pool`.
inline int32_t CompileProgram(const pxg_program& in, const int32_t* col_types, int ncols, DevProgram* out,
                              std::vector<uint8_t>* pool, size_t* pool_off) {
  std::memset(out, 0, sizeof(*out));
  if (in.n_insns <= 0 || in.n_insns > PXG_MAX_PROGRAM) return SetError(PXG_INVALID_ARGUMENT, "program length %d out of range", in.n_insns);
  if (!in.insns) return SetError(PXG_INVALID_ARGUMENT, "program has no instructions");
  std::vector<int> st;
  for (int pc = 0; pc < in.n_insns; ++pc) {
    const pxg_insn& x = in.insns[pc];
    const int op = x.op;
    switch (op) {
      case PXG_OP_COL:
        if (x.arg < 0 || x.arg >= ncols) return SetError(PXG_INVALID_ARGUMENT, "column %d out of range", x.arg);
        if (col_types && x.type != col_types[x.arg])
          return SetError(PXG_INVALID_ARGUMENT, "column %d has type %d, program expects %d", x.arg, col_types[x.arg], x.type);
        st.push_back(x.type);
        break;
      case PXG_OP_STATE_WORD:
        if (x.arg < 0 || x.arg >= ncols) return SetError(PXG_INVALID_ARGUMENT, "column %d out of range", x.arg);
        if (col_types && col_types[x.arg] != PXG_STRING)
          return SetError(PXG_INVALID_ARGUMENT, "state word of column %d, which is not STRING", x.arg);
        if (x.imm < 0 || !(x.type == PXG_INT64 || x.type == PXG_TIME64NS || x.type == PXG_FLOAT64))
          return SetError(PXG_INVALID_ARGUMENT, "bad state word (offset %lld, type %d)", (long long)x.imm, x.type);
        st.push_back(x.type);
        break;
      case PXG_OP_CONST:
        if ((x.type == PXG_STRING || x.type == PXG_UINT128) &&
            (x.arg < 0 || x.arg + (x.type == PXG_UINT128 ? 16 : x.imm) > in.pool_len || x.imm < 0))
          return SetError(PXG_INVALID_ARGUMENT, "constant outside pool");
        st.push_back(x.type);
        break;
      case PXG_OP_I2F: case PXG_OP_B2I: case PXG_OP_I2B: case PXG_OP_F2I: case PXG_OP_NEG_I: case PXG_OP_INV_I:
      case PXG_OP_NEG_F: case PXG_OP_NOT:
        if (st.empty()) return SetError(PXG_INVALID_ARGUMENT, "stack underflow at %d", pc);
        st.back() = x.type;
        break;
      default:
        if (!(IsFixedBinOp(op) || IsStrOp(op) || op == PXG_OP_EQ_U || op == PXG_OP_NE_U))
          return SetError(PXG_UNIMPLEMENTED, "opcode %d not supported", op);
        if (st.size() < 2) return SetError(PXG_INVALID_ARGUMENT, "stack underflow at %d", pc);
        if (IsStrOp(op) && (st[st.size() - 1] != PXG_STRING || st[st.size() - 2] != PXG_STRING))
          return SetError(PXG_INVALID_ARGUMENT, "string op on non-strings");
        st.pop_back();
        st.back() = x.type;
        break;
    }
    if (st.size() > PXG_MAX_STACK) return SetError(PXG_INVALID_ARGUMENT, "program stack deeper than %d", PXG_MAX_STACK);
    out->insns[pc].op = x.op;
    out->insns[pc].type = x.type;
    out->insns[pc].arg = x.arg;
    out->insns[pc].imm = x.imm;
  }
  if (st.size() != 1) return SetError(PXG_INVALID_ARGUMENT, "program leaves %zu values on the stack", st.size());
  if (st[0] != in.result_type) return SetError(PXG_INVALID_ARGUMENT, "program result type %d != declared %d", st[0], in.result_type);
  out->n = in.n_insns;
  out->result_type = in.result_type;
  *pool_off = pool->size();
  if (in.pool_len > 0) pool->insert(pool->end(), in.pool, in.pool + in.pool_len);
  while (pool->size() % 16) pool->push_back(0);
  // Fast shapes.
  const pxg_insn* I = in.insns;
  if (in.n_insns == 1 && I[0].op == PXG_OP_COL) {
    out->shape = kShapeCol;
    out->col = I[0].arg;
  } else if (in.n_insns == 3 && I[0].op == PXG_OP_COL && I[1].op == PXG_OP_CONST && IsFixedBinOp(I[2].op) &&
             I[0].type != PXG_STRING && I[0].type != PXG_UINT128 && I[1].type != PXG_STRING && I[1].type != PXG_UINT128) {
    out->shape = kShapeColOpConst;
    out->col = I[0].arg;
    out->conv = 0;
    out->binop = I[2].op;
    out->cimm = I[1].imm;
  } else if (in.n_insns == 4 && I[0].op == PXG_OP_COL && (I[1].op == PXG_OP_I2F || I[1].op == PXG_OP_B2I) &&
             I[2].op == PXG_OP_CONST && IsFixedBinOp(I[3].op) && I[0].type != PXG_STRING && I[0].type != PXG_UINT128 &&
             I[2].type != PXG_STRING && I[2].type != PXG_UINT128) {
    out->shape = kShapeColOpConst;
    out->col = I[0].arg;
    out->conv = I[1].op;
    out->binop = I[3].op;
    out->cimm = I[2].imm;
  } else {
    out->shape = kShapeGeneric;
  }
  return PXG_OK;
}

}  // namespace pxg
