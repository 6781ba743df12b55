// Device-side helpers shared by the MI355X state-engine kernels: typed column reads and the
// postfix predicate VM that replaces Siddhi's ExpressionExecutor trees.
//
// Semantics restated from the reference executors (C/ = modules/siddhi-core/src/main/java/io/siddhi/core/):
//   compare with a null operand -> false, except != -> true
//       (C/executor/condition/compare/CompareConditionExpressionExecutor.java:39-43,
//        .../compare/notequal/NotEqualCompareConditionExpressionExecutor.java:37)
//   numeric domains: Java binary promotion for > >= < <=; == / != on Float-Long in double
//       (.../compare/equal/EqualCompareConditionExpressionExecutorFloatLong.java:38); the lowering
//       (siddhi_amd/lowering.py::_cmp_domain) picks the domain per compare.
//   and: true iff both true; or: true iff either true; not: true unless operand is TRUE; is null
//       (C/executor/condition/{And,Or,Not,IsNull}ConditionExpressionExecutor.java)
#pragma once
#ifdef SG_HOST_ONLY
#include "sg_host_shim.h"
#else
#include <hip/hip_runtime.h>
#define SG_GLOBAL __attribute__((address_space(1)))
#endif
#include <stdint.h>
#include "../../include/siddhi_gpu.h"

// Column and packed-row reads go through global-address-space pointers: a generic pointer read out of a struct (a
// kernel-argument view, a descriptor) would make every access a flat load, which also waits on the LDS traffic of
// the same wave.
template <class T>
__device__ __forceinline__ const SG_GLOBAL T* gptr(const void* p) { return (const SG_GLOBAL T*)p; }

struct SgVal {
  int64_t i;
  double d;
  int type;
  int null;
};

struct SgCols {          // kernel-argument view of one batch's columns
  const void* col[SG_MAX_COLS];
  const uint8_t* nul[SG_MAX_COLS];
};

__device__ __forceinline__ SgVal sg_read_col(const SgCols& c, int col, int type, int64_t row) {
  SgVal v;
  v.type = type;
  v.i = 0;
  v.d = 0.0;
  v.null = (c.nul[col] != nullptr && gptr<uint8_t>(c.nul[col])[row]) ? 1 : 0;
  if (v.null) return v;
  switch (type) {
    case SG_T_LONG: v.i = gptr<int64_t>(c.col[col])[row]; break;
    case SG_T_FLOAT: v.d = (double)gptr<float>(c.col[col])[row]; break;
    case SG_T_DOUBLE: v.d = gptr<double>(c.col[col])[row]; break;
    default: v.i = gptr<int32_t>(c.col[col])[row]; break;
  }
  return v;
}

__device__ __forceinline__ int64_t sg_val_bits(const SgVal& v) {
  if (v.null) return 0;
  if (v.type == SG_T_FLOAT) {
    float f = (float)v.d;
    return (int64_t)(uint32_t)__float_as_uint(f);
  }
  if (v.type == SG_T_DOUBLE) return __double_as_longlong(v.d);
  return v.i;
}

__device__ __forceinline__ SgVal sg_val_from_bits(int64_t bits, int type, int null) {
  SgVal v;
  v.type = type;
  v.null = null;
  v.i = 0;
  v.d = 0.0;
  if (null) return v;
  if (type == SG_T_FLOAT) v.d = (double)__uint_as_float((uint32_t)bits);
  else if (type == SG_T_DOUBLE) v.d = __longlong_as_double(bits);
  else v.i = bits;
  return v;
}

__device__ __forceinline__ bool sg_cmp(int op, int dom, const SgVal& l, const SgVal& r) {
  if (op == 1) {
    if (l.null || r.null) return true;
  } else if (l.null || r.null) {
    return false;
  }
  if (dom == 3 || dom == 0) {  // dictionary ids / integral
    int64_t a = l.i, b = r.i;
    if (dom == 0) {  // int-vs-float handled by promotion domain, here both integral
      a = (l.type == SG_T_FLOAT || l.type == SG_T_DOUBLE) ? (int64_t)l.d : l.i;
      b = (r.type == SG_T_FLOAT || r.type == SG_T_DOUBLE) ? (int64_t)r.d : r.i;
    }
    switch (op) {
      case 0: return a == b;
      case 1: return a != b;
      case 2: return a > b;
      case 3: return a >= b;
      case 4: return a < b;
      default: return a <= b;
    }
  }
  if (dom == 1) {  // float domain
    float a = (l.type == SG_T_FLOAT || l.type == SG_T_DOUBLE) ? (float)l.d : (float)l.i;
    float b = (r.type == SG_T_FLOAT || r.type == SG_T_DOUBLE) ? (float)r.d : (float)r.i;
    switch (op) {
      case 0: return a == b;
      case 1: return a != b;
      case 2: return a > b;
      case 3: return a >= b;
      case 4: return a < b;
      default: return a <= b;
    }
  }
  double a = (l.type == SG_T_FLOAT || l.type == SG_T_DOUBLE) ? l.d : (double)l.i;
  double b = (r.type == SG_T_FLOAT || r.type == SG_T_DOUBLE) ? r.d : (double)r.i;
  switch (op) {
    case 0: return a == b;
    case 1: return a != b;
    case 2: return a > b;
    case 3: return a >= b;
    case 4: return a < b;
    default: return a <= b;
  }
}

// Java arithmetic of the math executors (C/executor/math/{add,subtract,multiply,divide,mod}/*ExpressionExecutor*.java):
// operands converted to the result type (ExpressionParser.parseArithmeticOperationResultType,
// C/util/parser/ExpressionParser.java:1413-1431); null operand -> null; / and % by zero -> null (int/long: right == 0;
// float/double: right == 0.0, so NaN divisors divide); int/long wrap two's complement; MIN / -1 = MIN, MIN % -1 = 0
// (JLS 15.17.2-3); float arithmetic in binary32, % is fmod (JLS 15.17.3).
__device__ __forceinline__ SgVal sg_math(int op, int rt, const SgVal& l, const SgVal& r) {
  SgVal o;
  o.type = rt;
  o.null = 0;
  o.i = 0;
  o.d = 0.0;
  if (l.null || r.null) { o.null = 1; return o; }
  auto as_d = [](const SgVal& v) { return (v.type == SG_T_FLOAT || v.type == SG_T_DOUBLE) ? v.d : (double)v.i; };
  if (rt == SG_T_DOUBLE) {
    double a = as_d(l), b = as_d(r);
    switch (op) {
      case 0: o.d = a + b; break;
      case 1: o.d = a - b; break;
      case 2: o.d = a * b; break;
      case 3: if (b == 0.0) o.null = 1; else o.d = a / b; break;
      default: if (b == 0.0) o.null = 1; else o.d = fmod(a, b); break;
    }
  } else if (rt == SG_T_FLOAT) {
    float a = (l.type == SG_T_FLOAT || l.type == SG_T_DOUBLE) ? (float)l.d : (float)l.i;
    float b = (r.type == SG_T_FLOAT || r.type == SG_T_DOUBLE) ? (float)r.d : (float)r.i;
    float c = 0.0f;
    switch (op) {
      case 0: c = a + b; break;
      case 1: c = a - b; break;
      case 2: c = a * b; break;
      case 3: if (b == 0.0f) o.null = 1; else c = a / b; break;
      default: if (b == 0.0f) o.null = 1; else c = fmodf(a, b); break;
    }
    o.d = (double)c;
  } else if (rt == SG_T_LONG) {
    uint64_t a = (uint64_t)l.i, b = (uint64_t)r.i;
    switch (op) {
      case 0: o.i = (int64_t)(a + b); break;
      case 1: o.i = (int64_t)(a - b); break;
      case 2: o.i = (int64_t)(a * b); break;
      case 3:
        if (r.i == 0) o.null = 1;
        else if (r.i == -1) o.i = (int64_t)(0 - a);
        else o.i = l.i / r.i;
        break;
      default:
        if (r.i == 0) o.null = 1;
        else if (r.i == -1) o.i = 0;
        else o.i = l.i % r.i;
        break;
    }
  } else {   // INT
    int32_t ai = (int32_t)l.i, bi = (int32_t)r.i;
    uint32_t a = (uint32_t)ai, b = (uint32_t)bi;
    int32_t c = 0;
    switch (op) {
      case 0: c = (int32_t)(a + b); break;
      case 1: c = (int32_t)(a - b); break;
      case 2: c = (int32_t)(a * b); break;
      case 3:
        if (bi == 0) o.null = 1;
        else if (bi == -1) c = (int32_t)(0u - a);
        else c = ai / bi;
        break;
      default:
        if (bi == 0) o.null = 1;
        else if (bi == -1) c = 0;
        else c = ai % bi;
        break;
    }
    o.i = c;
  }
  return o;
}

// Postfix VM. `Reader` supplies VAR operands: SgVal read(int state, int index_in_chain, int ret_slot, int type).
// Booleans are kept tri-state in SgVal (i = 0/1, null) so `not` of null is true (NotConditionExpressionExecutor).
// The operand stack is a private array indexed at run time (the compiler places it in scratch), or -- when the
// caller knows the program's depth (sg_prog_depth) -- D register slots addressed through unrolled selects, so the
// kernel has no private segment (k_pred).
#define SG_VM_STACK 16
template <int D>
struct SgArrStack {
  SgVal s[D];
  __host__ __device__ __forceinline__ SgVal get(int i) const { return s[i]; }
  __host__ __device__ __forceinline__ void set(int i, const SgVal& v) { s[i] = v; }
};
#if defined(__clang__)   // (ext_vector_type; the g++ host harness never instantiates it)
template <int D>
struct SgRegStack {   // one register vector per field: run-time indices become register moves, not scratch
  typedef int64_t VI __attribute__((ext_vector_type(D)));
  typedef double VD __attribute__((ext_vector_type(D)));
  typedef int32_t VT __attribute__((ext_vector_type(D)));
  VI i;
  VD d;
  VT tn;   // type | null << 16
  __host__ __device__ __forceinline__ SgVal get(int k) const {
    SgVal v;
    v.i = i[k];
    v.d = d[k];
    const int32_t x = tn[k];
    v.type = x & 0xffff;
    v.null = x >> 16;
    return v;
  }
  __host__ __device__ __forceinline__ void set(int k, const SgVal& v) {
    i[k] = v.i;
    d[k] = v.d;
    tn[k] = (v.type & 0xffff) | (v.null << 16);
  }
};
#endif
template <class Reader, class Stack = SgArrStack<SG_VM_STACK>>
__device__ __forceinline__ bool sg_run(const int64_t* code, int len, Reader& rd, SgVal& top) {
  Stack st;
  int sp = 0;
  int pc = 0;
  while (pc < len) {
    int op = (int)code[pc];
    switch (op) {
      case SG_OP_VAR: {
        st.set(sp++, rd.read((int)code[pc + 1], (int)code[pc + 2], (int)code[pc + 3], (int)code[pc + 4]));
        pc += 5;
        break;
      }
      case SG_OP_CONST: {
        st.set(sp++, sg_val_from_bits(code[pc + 2], (int)code[pc + 1], 0));
        pc += 3;
        break;
      }
      case SG_OP_CMP: {
        SgVal r = st.get(--sp);
        SgVal l = st.get(--sp);
        SgVal o;
        o.type = SG_T_BOOL;
        o.null = 0;
        o.d = 0;
        o.i = sg_cmp((int)code[pc + 1], (int)code[pc + 2], l, r) ? 1 : 0;
        st.set(sp++, o);
        pc += 3;
        break;
      }
      case SG_OP_AND:
      case SG_OP_OR: {
        SgVal r = st.get(--sp);
        SgVal l = st.get(--sp);
        bool lt = !l.null && l.i, rt = !r.null && r.i;
        SgVal o;
        o.type = SG_T_BOOL;
        o.null = 0;
        o.d = 0;
        o.i = (op == SG_OP_AND) ? (lt && rt) : (lt || rt);
        st.set(sp++, o);
        pc += 1;
        break;
      }
      case SG_OP_NOT: {
        SgVal x = st.get(sp - 1);
        x.i = !(!x.null && x.i);
        x.null = 0;
        x.type = SG_T_BOOL;
        st.set(sp - 1, x);
        pc += 1;
        break;
      }
      case SG_OP_ISNULL: {
        SgVal x = st.get(sp - 1);
        x.i = x.null ? 1 : 0;
        x.null = 0;
        x.type = SG_T_BOOL;
        st.set(sp - 1, x);
        pc += 1;
        break;
      }
      case SG_OP_MATH: {
        SgVal r = st.get(--sp);
        SgVal l = st.get(--sp);
        st.set(sp++, sg_math((int)code[pc + 1], (int)code[pc + 2], l, r));
        pc += 3;
        break;
      }
      default:
        return false;
    }
  }
  if (sp <= 0) return false;
  top = st.get(sp - 1);
  return true;
}

template <class Reader, class Stack = SgArrStack<SG_VM_STACK>>
__device__ __forceinline__ bool sg_eval(const int64_t* code, int len, Reader& rd) {
  if (len <= 0) return true;
  SgVal top;
  if (!sg_run<Reader, Stack>(code, len, rd, top)) return false;
  return !top.null && top.i != 0;
}

// Largest operand-stack depth of a postfix program (host side; 1 << 30 for an unknown opcode).
static inline int sg_prog_depth(const int64_t* code, int len) {
  int sp = 0, mx = 0, pc = 0;
  while (pc < len) {
    switch ((int)code[pc]) {
      case SG_OP_VAR: ++sp; pc += 5; break;
      case SG_OP_CONST: ++sp; pc += 3; break;
      case SG_OP_CMP: case SG_OP_MATH: --sp; pc += 3; break;
      case SG_OP_AND: case SG_OP_OR: --sp; pc += 1; break;
      case SG_OP_NOT: case SG_OP_ISNULL: pc += 1; break;
      default: return 1 << 30;
    }
    mx = sp > mx ? sp : mx;
  }
  return mx;
}
