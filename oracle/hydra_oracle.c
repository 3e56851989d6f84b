/*
 * oracle/hydra_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's bucket-reduction hot path, used as the checker by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  It is never linked into,
 * called by, or substituted for the product (hydra_amd/libhydra_hip.so).
 *
 * Pinned against: tests/golden/*.npz, produced by oracle/gen_golden.py from the reference itself
 * (oracle/_ref/libgloo_ref.so, compiled from /root/reference/gloo sources by oracle/Makefile),
 * and against the reference's own known-answer tests (tests/test_oracle.py).
 *
 * What is restated (reference file:line):
 *   orc_op            gloo::sum/product/max/min<T>      gloo/gloo/math.h:15-73
 *   f16 conversions   cpu_float2half_rn/cpu_half2float  gloo/gloo/types.h:207-320
 *   orc_ring_plan     segment geometry of ring()        gloo/gloo/allreduce.cc:199-221
 *   orc_allreduce     local reduce + ring RS/AG result  gloo/gloo/allreduce.cc:46-146, 147-422
 *   orc_split_aa/_ag  bew_allreduce_a rail split        gloo/gloo/pipeallreduce-a.h:137-376
 *   orc_reduce        gloo::reduce root result         gloo/gloo/reduce.cc:21-262
 * bf16 (dtype 9) has no reference counterpart: c = bf16_rne(float(a) + float(b)) (our spec).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { D_INT8 = 0, D_UINT8, D_INT32, D_UINT32, D_INT64, D_UINT64, D_FLOAT32, D_FLOAT64,
       D_FLOAT16, D_BFLOAT16 };
enum { OP_SUM = 0, OP_PRODUCT = 1, OP_MAX = 2, OP_MIN = 3 };

size_t orc_esize(int dtype) {
  static const size_t sz[] = {1, 1, 4, 4, 8, 8, 4, 8, 2, 2};
  return (dtype >= 0 && dtype <= 9) ? sz[dtype] : 0;
}

/* ---- fp16 exactly as gloo/gloo/types.h:207-320 (RNE, NaN -> 0x7fff / 0x7fffffff) ---- */
uint16_t orc_f2h(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  uint32_t u = x & 0x7fffffffu, sign, exponent, mantissa, shift, lsb, lsb_s1, lsb_m1, rem;
  if (u > 0x7f800000u) return 0x7fffu;
  sign = (x >> 16) & 0x8000u;
  if (u > 0x477fefffu) return (uint16_t)(sign | 0x7c00u);
  if (u < 0x33000001u) return (uint16_t)sign;
  exponent = (u >> 23) & 0xffu;
  mantissa = u & 0x7fffffu;
  if (exponent > 0x70u) {
    shift = 13;
    exponent -= 0x70u;
  } else {
    shift = 0x7eu - exponent;
    exponent = 0;
    mantissa |= 0x800000u;
  }
  lsb = 1u << shift;
  lsb_s1 = lsb >> 1;
  lsb_m1 = lsb - 1;
  rem = mantissa & lsb_m1;
  mantissa >>= shift;
  if (rem > lsb_s1 || (rem == lsb_s1 && (mantissa & 1u))) {
    ++mantissa;
    if (!(mantissa & 0x3ffu)) {
      ++exponent;
      mantissa = 0;
    }
  }
  return (uint16_t)(sign | (exponent << 10) | mantissa);
}

float orc_h2f(uint16_t h) {
  uint32_t sign = (h >> 15) & 1u, exponent = (h >> 10) & 0x1fu, mantissa = (uint32_t)(h & 0x3ffu) << 13;
  if (exponent == 0x1fu) {
    if (mantissa) { sign = 0; mantissa = 0x7fffffu; }
    exponent = 0xffu;
  } else if (!exponent) {
    if (mantissa) {
      uint32_t msb;
      exponent = 0x71u;
      do {
        msb = mantissa & 0x400000u;
        mantissa <<= 1;
        --exponent;
      } while (!msb);
      mantissa &= 0x7fffffu;
    }
  } else {
    exponent += 0x70u;
  }
  uint32_t t = (sign << 31) | (exponent << 23) | mantissa;
  float f;
  memcpy(&f, &t, 4);
  return f;
}

/* bf16: round-to-nearest-even from fp32, NaN kept a (quiet) NaN. */
uint16_t orc_f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float orc_bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

/* ---- element-wise ops: math.h:15-73.  max/min keep std::max/std::min operand semantics:
 *      std::max(a,b) = (a < b) ? b : a ;  std::min(a,b) = (b < a) ? b : a.               ---- */
#define DEF_OPS(NAME, T)                                                                  \
  static void NAME(int op, T* c, const T* a, const T* b, size_t n) {                      \
    size_t i;                                                                             \
    switch (op) {                                                                         \
      case OP_SUM: for (i = 0; i < n; i++) c[i] = (T)(a[i] + b[i]); break;                \
      case OP_PRODUCT: for (i = 0; i < n; i++) c[i] = (T)(a[i] * b[i]); break;            \
      case OP_MAX: for (i = 0; i < n; i++) c[i] = (a[i] < b[i]) ? b[i] : a[i]; break;     \
      case OP_MIN: for (i = 0; i < n; i++) c[i] = (b[i] < a[i]) ? b[i] : a[i]; break;     \
    }                                                                                     \
  }
DEF_OPS(ops_f32, float)
DEF_OPS(ops_f64, double)

/* Integer ops wrap modulo 2^bits (the reference's C++ int8/16 promotion + narrowing does this;
 * for int32/int64 overflow is UB in the reference, fixtures stay in range). */
#define DEF_IOPS(NAME, T, U)                                                              \
  static void NAME(int op, T* c, const T* a, const T* b, size_t n) {                      \
    size_t i;                                                                             \
    switch (op) {                                                                         \
      case OP_SUM: for (i = 0; i < n; i++) c[i] = (T)((U)a[i] + (U)b[i]); break;          \
      case OP_PRODUCT: for (i = 0; i < n; i++) c[i] = (T)((U)a[i] * (U)b[i]); break;      \
      case OP_MAX: for (i = 0; i < n; i++) c[i] = (a[i] < b[i]) ? b[i] : a[i]; break;     \
      case OP_MIN: for (i = 0; i < n; i++) c[i] = (b[i] < a[i]) ? b[i] : a[i]; break;     \
    }                                                                                     \
  }
DEF_IOPS(ops_i8, int8_t, uint32_t)
DEF_IOPS(ops_u8, uint8_t, uint32_t)
DEF_IOPS(ops_i32, int32_t, uint32_t)
DEF_IOPS(ops_u32, uint32_t, uint32_t)
DEF_IOPS(ops_i64, int64_t, uint64_t)
DEF_IOPS(ops_u64, uint64_t, uint64_t)

/* float16: every op converts to fp32, computes, converts back (types.h:163-228) -- and every
 * store goes through float16::operator= (types.h:112-118), whose guard `if (rhs != *this)`
 * resolves to rhs.x == cpu_float2half_rn((float)this->x) (operator!= -> operator==(const int&),
 * types.h:123-130): the store is SKIPPED when the new bits equal the half of the old bits read
 * as an integer.  operator+ stores twice (result = lhs; result += rhs: types.h:196-200), then
 * c[i] = result stores into c.  So the output depends on c's previous bits; in the ring c == a. */
static uint16_t f16_assign(uint16_t old_bits, uint16_t new_bits) {
  return (new_bits == orc_f2h((float)old_bits)) ? old_bits : new_bits;
}

static void ops_f16(int op, uint16_t* c, const uint16_t* a, const uint16_t* b, size_t n) {
  for (size_t i = 0; i < n; i++) {
    uint16_t L = a[i], R = b[i], C0 = c[i], res = 0;
    float x = orc_h2f(L), y = orc_h2f(R);
    switch (op) {
      case OP_SUM: res = f16_assign(L, orc_f2h(x + y)); break;
      case OP_PRODUCT: res = f16_assign(L, orc_f2h(x * y)); break;
      case OP_MAX: res = (x < y) ? R : L; break;
      case OP_MIN: res = (y < x) ? R : L; break;
    }
    c[i] = f16_assign(C0, res);
  }
}

static void ops_bf16(int op, uint16_t* c, const uint16_t* a, const uint16_t* b, size_t n) {
  for (size_t i = 0; i < n; i++) {
    float x = orc_bf2f(a[i]), y = orc_bf2f(b[i]);
    switch (op) {
      case OP_SUM: c[i] = orc_f2bf(x + y); break;
      case OP_PRODUCT: c[i] = orc_f2bf(x * y); break;
      case OP_MAX: c[i] = (x < y) ? b[i] : a[i]; break;
      case OP_MIN: c[i] = (y < x) ? b[i] : a[i]; break;
    }
  }
}

/* c[i] = op(a[i], b[i]);  c may alias a or b exactly (element-wise, forward order). */
int orc_op(int op, int dtype, void* c, const void* a, const void* b, size_t n) {
  switch (dtype) {
    case D_INT8: ops_i8(op, c, a, b, n); return 0;
    case D_UINT8: ops_u8(op, c, a, b, n); return 0;
    case D_INT32: ops_i32(op, c, a, b, n); return 0;
    case D_UINT32: ops_u32(op, c, a, b, n); return 0;
    case D_INT64: ops_i64(op, c, a, b, n); return 0;
    case D_UINT64: ops_u64(op, c, a, b, n); return 0;
    case D_FLOAT32: ops_f32(op, c, a, b, n); return 0;
    case D_FLOAT64: ops_f64(op, c, a, b, n); return 0;
    case D_FLOAT16: ops_f16(op, c, a, b, n); return 0;
    case D_BFLOAT16: ops_bf16(op, c, a, b, n); return 0;
  }
  return 1;
}

/* Mixed precision accumulate (BASELINE config 5, no reference counterpart):
 * acc_f32[i] = acc_f32[i] + float(b_bf16[i]). */
void orc_acc_bf16_f32(float* acc, const uint16_t* b, size_t n) {
  for (size_t i = 0; i < n; i++) acc[i] = acc[i] + orc_bf2f(b[i]);
}

/* ---- ring geometry, allreduce.cc:199-221 ---- */
static size_t round_up(size_t v, size_t m) { size_t r = v % m; return r ? v + m - r : v; }

void orc_ring_plan(int P, size_t n, size_t esize, size_t max_segment, size_t* num_segments,
                   size_t* segment_bytes, size_t* segments_per_rank) {
  size_t total = n * esize;
  size_t per = max_segment / esize;
  size_t max_seg_bytes = esize * (per > 1 ? per : 1);
  size_t want = (total + max_seg_bytes - 1) / max_seg_bytes;
  if (want < (size_t)P * 2) want = (size_t)P * 2;
  size_t ns = round_up(want, (size_t)P);
  *num_segments = ns;
  *segments_per_rank = ns / (size_t)P;
  *segment_bytes = round_up((total + ns - 1) / ns, esize);
}

/* ---- allreduce result, allreduce.cc:46-422 ----
 * ranks: P, each with nptr output buffers (and nptr inputs when in != NULL), layout [rank][ptr].
 * Local reduce (genLocalReduceFunction, :46-83):
 *   1 input      -> x_r = in[0]
 *   >=2 inputs   -> x_r = op(op(in0,in1),in2)...
 *   no inputs    -> x_r = op(op(out0,out1),out2)...
 * Ring fold (reduce-scatter, :284-344; recv from rank+1, send to rank-1; c = op(local, recv)):
 *   segment k is owned by rank q = k / S and ends as
 *   op(x_q, op(x_{q+1}, ... op(x_{q-2}, x_{q-1})))   (indices mod P)
 * All-gather + genLocalBroadcastFunction then copy that into every output of every rank.
 * P == 1 short-circuits to local reduce + broadcast (:129-133).                           */
/* Each rank's locally reduced value x_r (allreduce.cc:46-97): out[0] op= the other inputs. */
static void local_values(int P, int nptr, int op, int dtype, size_t n, void** in, void** out,
                         unsigned char* x) {
  size_t bytes = n * orc_esize(dtype);
  for (int r = 0; r < P; r++) {
    unsigned char* xr = x + (size_t)r * bytes;
    void** src = in ? in + r * nptr : out + r * nptr;
    if (in && nptr == 1) {
      memcpy(xr, src[0], bytes);
    } else {
      if (in) {
        /* fn(out0, in0, in1): out0's old bits matter for float16 stores (see ops_f16) */
        memcpy(xr, out[r * nptr], bytes);
        orc_op(op, dtype, xr, src[0], src[1], n);
        for (int i = 2; i < nptr; i++) orc_op(op, dtype, xr, xr, src[i], n);
      } else {
        memcpy(xr, src[0], bytes);
        for (int i = 1; i < nptr; i++) orc_op(op, dtype, xr, xr, src[i], n);
      }
    }
  }
}

int orc_allreduce(int P, int nptr, int op, int dtype, size_t n, void** in, void** out,
                  size_t max_segment) {
  size_t es = orc_esize(dtype);
  if (!es || P < 1 || nptr < 1) return 1;
  size_t bytes = n * es;
  unsigned char* x = (unsigned char*)malloc(bytes * (size_t)P + 1);
  unsigned char* acc = (unsigned char*)malloc(bytes + 1);
  if (!x || !acc) { free(x); free(acc); return 2; }
  local_values(P, nptr, op, dtype, n, in, out, x);
  if (P == 1) {
    memcpy(acc, x, bytes);
  } else {
    size_t ns, sb, S;
    orc_ring_plan(P, n, es, max_segment ? max_segment : (1u << 20), &ns, &sb, &S);
    unsigned char* tmp = (unsigned char*)malloc(sb + 1);
    if (!tmp) { free(x); free(acc); return 2; }
    for (size_t k = 0; k < ns; k++) {
      size_t off = k * sb;
      if (off >= bytes) break;
      size_t len = (bytes - off < sb) ? bytes - off : sb;
      size_t cnt = len / es;
      int q = (int)(k / S);
      /* start with x_{q-1}, fold leftwards: acc = op(x_j, acc) for j = q-2, ..., q, each
       * computed in place on a copy of the local x_j, as the ring does (c == a == local). */
      memcpy(acc + off, x + (size_t)((q + P - 1) % P) * bytes + off, len);
      for (int d = P - 2; d >= 0; d--) {
        int j = (q + d) % P;
        memcpy(tmp, x + (size_t)j * bytes + off, len);
        orc_op(op, dtype, tmp, tmp, acc + off, cnt);
        memcpy(acc + off, tmp, len);
      }
    }
    free(tmp);
  }
  for (int r = 0; r < P; r++)
    for (int i = 0; i < nptr; i++) memcpy(out[r * nptr + i], acc, bytes);
  free(x);
  free(acc);
  return 0;
}

/* ---- BCUBE (allreduce.cc:423-700) ----
 * Group sizes: factors of 2 while P divides, then the remainder (computeGroupSizePerStep,
 * :426-437).  Step s: rank r's group is the ranks base + i*dist (i < g); the current buffer
 * range splits into g chunks of ceil(len/g); r keeps chunk (r/dist) % g and folds the group's
 * partials into it in place, own value first, then peers in group order (:592-603).  After the
 * last step every element has one owner; the all-gather copies the owner's bits everywhere. */
int orc_allreduce_bcube(int P, int nptr, int op, int dtype, size_t n, void** in, void** out) {
  size_t es = orc_esize(dtype);
  if (!es || P < 1 || nptr < 1) return 1;
  size_t bytes = n * es;
  unsigned char* x = (unsigned char*)malloc(bytes * (size_t)P + 1);   /* partials */
  unsigned char* snap = (unsigned char*)malloc(bytes * (size_t)P + 1);
  size_t* boff = (size_t*)calloc((size_t)P, sizeof(size_t));          /* buffer range per rank */
  size_t* blen = (size_t*)calloc((size_t)P, sizeof(size_t));
  if (!x || !snap || !boff || !blen) { free(x); free(snap); free(boff); free(blen); return 2; }
  local_values(P, nptr, op, dtype, n, in, out, x);
  size_t sizes[64];
  int steps = 0;
  {
    size_t sz = (size_t)P;
    while (sz % 2 == 0) { sizes[steps++] = 2; sz /= 2; }
    if (sz > 1) sizes[steps++] = sz;
  }
  for (int r = 0; r < P; r++) { boff[r] = 0; blen[r] = n; }
  size_t dist = 1;
  for (int s = 0; s < steps; s++) {
    size_t g = sizes[s];
    memcpy(snap, x, bytes * (size_t)P);
    size_t* noff = (size_t*)malloc((size_t)P * sizeof(size_t));
    size_t* nlen = (size_t*)malloc((size_t)P * sizeof(size_t));
    for (int r = 0; r < P; r++) {
      size_t grank = ((size_t)r / dist) % g, base = (size_t)r - grank * dist;
      size_t chunk = (blen[r] + g - 1) / g;
      size_t moff = boff[r] + grank * chunk;
      size_t mlen = blen[r] > grank * chunk ? blen[r] - grank * chunk : 0;
      if (mlen > chunk) mlen = chunk;
      unsigned char* mine = x + (size_t)r * bytes + moff * es;
      for (size_t i = 0; i < g; i++) {
        size_t peer = base + i * dist;
        if (peer == (size_t)r || mlen == 0) continue;
        orc_op(op, dtype, mine, mine, snap + peer * bytes + moff * es, mlen);
      }
      noff[r] = moff;
      nlen[r] = mlen;
    }
    memcpy(boff, noff, (size_t)P * sizeof(size_t));
    memcpy(blen, nlen, (size_t)P * sizeof(size_t));
    free(noff);
    free(nlen);
    dist *= g;
  }
  /* all-gather: every element's owner (the rank whose final range holds it) supplies the bits */
  unsigned char* res = snap;
  if (P == 1) memcpy(res, x, bytes);
  for (int r = 0; r < P && P > 1; r++)
    if (blen[r]) memcpy(res + boff[r] * es, x + (size_t)r * bytes + boff[r] * es, blen[r] * es);
  for (int r = 0; r < P; r++)
    for (int i = 0; i < nptr; i++) memcpy(out[r * nptr + i], res, bytes);
  free(x);
  free(snap);
  free(boff);
  free(blen);
  return 0;
}

/* ---- bew_allreduce_a rail split, pipeallreduce-a.h:296-376 (AA, default) and :137-294 (AG,
 *      env ALLREDUCE_GLEX).  e1 -> rail 1 (opts3/context), e2 -> rail 2 (opts2/context2).   ---- */
static void split_finish(size_t n, int cout_ele, int w_2, size_t* e1, size_t* e2) {
  int cout_mode = (int)(n % (size_t)cout_ele);
  if (cout_mode == 0) *e2 = (size_t)w_2 * n / (size_t)cout_ele;
  else *e2 = (size_t)w_2 * (n - (size_t)cout_mode) / (size_t)cout_ele;
  *e1 = n - *e2;
}

void orc_split_aa(int P, size_t n, size_t* e1, size_t* e2) {
  int ce, w;
  if (P == 2) {
    if (n < 65536) { ce = 1; w = 1; }
    else if (1048576 < n && n < 2097153) { ce = 100; w = 48; }
    else { ce = 2; w = 1; }
  } else if (P == 3) {
    if (n < 131072) { ce = 1; w = 1; } else { ce = 2; w = 1; }
  } else if (P == 4) {
    if (n < 65537) { ce = 1; w = 1; }
    else if (524287 < n && n < 16777217) { ce = 100; w = 52; }
    else { ce = 2; w = 1; }
  } else if (P == 6) {
    if (n < 65537) { ce = 1; w = 1; } else { ce = 2; w = 1; }
  } else {
    if (n < 131072) { ce = 1; w = 1; } else { ce = 2; w = 1; }
  }
  split_finish(n, ce, w, e1, e2);
}

void orc_split_ag(int P, size_t n, size_t* e1, size_t* e2) {
  int ce = 1, w = 1;
  if (P == 2) {
    ce = 100;
    if (n < 262145) { ce = 1; w = 1; }
    else if (262144 < n && n < 524289) { ce = 1; w = 1; }
    else if (524288 < n && n < 1048577) w = 75;
    else if (1048576 < n && n < 2097153) w = 74;
    else if (2097152 < n && n < 4194305) w = 72;
    else if (4194304 < n && n < 8388609) w = 69;
    else if (8388608 < n && n < 16777217) w = 67;
    else if (16777216 < n && n < 33554433) w = 65;
    else if (33554432 < n && n < 67108865) w = 65;
    else w = 60;
  } else if (P == 3) {
    ce = 100;
    if (n < 524289) { ce = 1; w = 1; }
    else if (524288 < n && n < 1048577) w = 80;
    else if (1048576 < n && n < 2097153) { ce = 15; w = 11; }
    else if (2097152 < n && n < 4194305) w = 70;
    else if (4194304 < n && n < 8388609) w = 68;
    else if (8388608 < n && n < 16777217) w = 64;
    else if (16777216 < n && n < 33554433) w = 65;
    else if (8388608 < n && n < 67108865) w = 64;
    else { ce = 2; w = 1; }
  } else if (P == 4) {
    ce = 100;
    if (n < 828344) { ce = 1; w = 1; }
    else if (828343 < n && n < 1048577) w = 81;
    else if (1048576 < n && n < 2097153) w = 73;
    else if (2097152 < n && n < 4194305) w = 70;
    else if (4194304 < n && n < 8388609) w = 67;
    else if (8388608 < n && n < 16777217) w = 65;
    else if (16777216 < n && n < 33554433) w = 65;
    else if (33554432 < n && n < 67108865) w = 66;
    else { ce = 2; w = 1; }
  } else if (P == 6) {
    ce = 100;
    if (n < 1048577) { ce = 1; w = 1; }
    else if (1048576 < n && n < 2097153) w = 73;
    else if (2097152 < n && n < 4194305) w = 70;
    else if (4194304 < n && n < 8388609) w = 66;
    else if (8388608 < n && n < 16777217) w = 66;
    else if (16777216 < n && n < 33554433) w = 64;
    else if (33554432 < n && n < 67108865) w = 66;
    else { ce = 2; w = 1; }
  } else {
    if (n < 6145) { ce = 1; w = 0; }
    else { ce = 1; w = 1; }
  }
  split_finish(n, ce, w, e1, e2);
}

/* ---- AllreduceOptions::Func-shaped entry points (void(void*, const void*, const void*, size_t),
 *      gloo/gloo/allreduce.h:36) so host-runtime tests can plug the oracle in as the reducer. ---- */
void orc_sum_f32(void* c, const void* a, const void* b, size_t n) { orc_op(OP_SUM, D_FLOAT32, c, a, b, n); }
void orc_sum_i32(void* c, const void* a, const void* b, size_t n) { orc_op(OP_SUM, D_INT32, c, a, b, n); }
void orc_sum_u64(void* c, const void* a, const void* b, size_t n) { orc_op(OP_SUM, D_UINT64, c, a, b, n); }
void orc_sum_f16(void* c, const void* a, const void* b, size_t n) { orc_op(OP_SUM, D_FLOAT16, c, a, b, n); }

/* ---- old-style AllreduceRing<T> (gloo/gloo/allreduce_ring.h:71-106) ----
 * bufs: P*nptr pointers [rank][ptr], in place.  Per rank: ptrs[0] = op(ptrs[0], ptrs[i]) for
 * i >= 1 (in place); then P-1 rounds each folding the raw local value of the next rank to the
 * LEFT: acc = op(acc, x_{r-k}) for k = 1..P-1 (c == a == acc); then ptrs[i] = ptrs[0].
 * Unlike the new-style ring, every rank ends with its own fold order. */
int orc_allreduce_ring_old(int P, int nptr, int op, int dtype, size_t n, void** bufs) {
  size_t es = orc_esize(dtype);
  if (!es || P < 1 || nptr < 1) return 1;
  size_t bytes = n * es;
  unsigned char* x = (unsigned char*)malloc(bytes * (size_t)P + 1);
  if (!x) return 2;
  for (int r = 0; r < P; r++) {
    void* p0 = bufs[r * nptr];
    for (int i = 1; i < nptr; i++) orc_op(op, dtype, p0, p0, bufs[r * nptr + i], n);
    memcpy(x + (size_t)r * bytes, p0, bytes);
  }
  for (int r = 0; r < P; r++) {
    void* p0 = bufs[r * nptr];
    for (int k = 1; k < P; k++)
      orc_op(op, dtype, p0, p0, x + (size_t)((r - k + P) % P) * bytes, n);
    for (int i = 1; i < nptr; i++) memcpy(bufs[r * nptr + i], p0, bytes);
  }
  free(x);
  return 0;
}
/* ---- AllreduceRingChunked<T> (gloo/gloo/allreduce_ring_chunked.h:77-200) ----
 * 2P chunks of max(256, ceil(n/2P)) elements (:32-36).  Rank s seeds chunks 2s and 2s+1
 * (:88-89); each of the next P-1 ranks folds its own value in place, local op inbox (:138-139),
 * so chunk c (s = c/2) ends as x_{s-1} op (x_{s-2} op (... op (x_{s+1} op x_s))), which the
 * broadcast pass then copies to every rank (:146-186). */
int orc_allreduce_ring_chunked(int P, int nptr, int op, int dtype, size_t n, void** bufs) {
  size_t es = orc_esize(dtype);
  if (!es || P < 1 || nptr < 1) return 1;
  for (int r = 0; r < P; r++) {
    void* p0 = bufs[r * nptr];
    for (int i = 1; i < nptr; i++) orc_op(op, dtype, p0, p0, bufs[r * nptr + i], n);
  }
  if (P > 1) {
    size_t chunks = 2 * (size_t)P;
    size_t ce = (n + chunks - 1) / chunks;
    if (ce < 256) ce = 256;
    unsigned char* acc = (unsigned char*)malloc(ce * es + 1);
    unsigned char* loc = (unsigned char*)malloc(ce * es + 1);
    if (!acc || !loc) { free(acc); free(loc); return 2; }
    for (size_t c = 0; c < chunks; c++) {
      size_t off = c * ce;
      if (off >= n) break;
      size_t len = n - off < ce ? n - off : ce;
      int s = (int)(c / 2);
      memcpy(acc, (unsigned char*)bufs[s * nptr] + off * es, len * es);
      for (int d = 1; d < P; d++) {
        int q = (s + d) % P;
        memcpy(loc, (unsigned char*)bufs[q * nptr] + off * es, len * es);
        orc_op(op, dtype, loc, loc, acc, len); /* the ring hop: local = local op inbox */
        memcpy(acc, loc, len * es);
      }
      for (int r = 0; r < P; r++) memcpy((unsigned char*)bufs[r * nptr] + off * es, acc, len * es);
    }
    free(acc);
    free(loc);
  }
  for (int r = 0; r < P; r++)
    for (int i = 1; i < nptr; i++) memcpy(bufs[r * nptr + i], bufs[r * nptr], n * es);
  return 0;
}

/* ---- AllreduceHalvingDoubling<T> (gloo/gloo/allreduce_halving_doubling.h:37-358) ----
 * steps = floor(log2 P), 2^steps chunks of ceil(n / 2^steps) elements (:76-78).  Ranks form
 * binary blocks, the largest first (:39-64).  Inside a block: recursive-halving reduce-scatter
 * (step i exchanges with rank ^ 2^i, local op= received, :241-256), then recursive-doubling
 * allgather (:316-338).  Between blocks: each rank folds the piece its smaller-block partner
 * sends (:263-269), scatters its reduced chunk to the next larger block in bit-reversed order
 * (:273-287), takes the larger block's finished pieces back (:293-301) and forwards its chunk to
 * the smaller block (:306-313).  Restated as a phase-ordered simulation: the schedule's only
 * cross-rank dependencies are those messages, so applying them block by block in that order
 * yields the reference's bits. */
typedef struct {
  uint32_t off, size, steps, rib, smaller, larger;
  size_t send_off[32], recv_off[32], send_cnt[32], recv_cnt[32];
  size_t sc_larger; /* sendCountToLargerBlock_ (:195-196) */
} hd_rank;

static uint32_t hd_log2(uint64_t x) { uint32_t l = 0; while (x >>= 1) l++; return l; }

static uint32_t hd_rev(uint32_t ctr, uint32_t nbits) { /* reverseLastNBits (:23-34) */
  uint32_t r = 0;
  for (uint32_t b = 0; b < nbits; b++) r = (r << 1) | ((ctr >> b) & 1u);
  return r;
}

static void hd_geometry(int P, int rank, size_t n, hd_rank* g) {
  const uint32_t steps = hd_log2((uint64_t)P);
  const size_t chunk = (n + ((size_t)1 << steps) - 1) >> steps;
  memset(g, 0, sizeof *g);
  uint32_t off = (uint32_t)P, bs = 1, cur = 0, prev = 0;
  do { /* initBinaryBlocks (:39-64) */
    if ((uint32_t)P & bs) {
      prev = cur;
      cur = bs;
      off -= bs;
      if (g->size) { g->larger = cur; break; }
      if (off <= (uint32_t)rank) { g->off = off; g->size = cur; g->smaller = prev; }
    }
    bs <<= 1;
  } while (off != 0);
  g->steps = hd_log2(g->size);
  g->rib = (uint32_t)rank % g->size;
  size_t step_chunk = steps ? chunk << (steps - 1) : 0, base = 0;
  for (uint32_t i = 0; i < g->steps; i++) { /* :113-157 */
    const uint32_t bit = 1u << i, dest = (uint32_t)rank ^ bit;
    g->send_off[i] = base + ((dest & bit) ? step_chunk : 0);
    g->recv_off[i] = base + (((uint32_t)rank & bit) ? step_chunk : 0);
    if (g->send_off[i] < n) g->send_cnt[i] = n - g->send_off[i] < step_chunk ? n - g->send_off[i] : step_chunk;
    if (g->recv_off[i] < n) g->recv_cnt[i] = n - g->recv_off[i] < step_chunk ? n - g->recv_off[i] : step_chunk;
    if ((uint32_t)rank & bit) base += step_chunk;
    step_chunk >>= 1;
  }
  if (g->larger) g->sc_larger = step_chunk >> (hd_log2(g->larger / g->size) - 1);
}

int orc_allreduce_halving_doubling(int P, int nptr, int op, int dtype, size_t n, void** bufs) {
  size_t es = orc_esize(dtype);
  if (!es || P < 1 || nptr < 1) return 1;
  for (int r = 0; r < P; r++) {
    void* p0 = bufs[r * nptr];
    for (int i = 1; i < nptr; i++) orc_op(op, dtype, p0, p0, bufs[r * nptr + i], n);
  }
  int rc = 0;
  if (P > 1 && n > 0) {
    hd_rank* g = (hd_rank*)calloc((size_t)P, sizeof(hd_rank));
    unsigned char* snap = (unsigned char*)malloc((size_t)P * n * es);
    if (!g || !snap) { free(g); free(snap); return 2; }
#define B(r) ((unsigned char*)bufs[(r) * nptr])
#define SNAP(r) (snap + (size_t)(r) * n * es)
    uint32_t max_steps = 0;
    for (int r = 0; r < P; r++) {
      hd_geometry(P, r, n, &g[r]);
      if (g[r].steps > max_steps) max_steps = g[r].steps;
    }
    /* 1. reduce-scatter inside every block */
    for (uint32_t i = 0; i < max_steps; i++) {
      for (int r = 0; r < P; r++) memcpy(SNAP(r), B(r), n * es);
      for (int r = 0; r < P; r++) {
        if (g[r].steps <= i || !g[r].recv_cnt[i]) continue;
        const int q = r ^ (1 << i);
        if (g[q].send_cnt[i] != g[r].recv_cnt[i]) { rc = 3; goto out; }
        orc_op(op, dtype, B(r) + g[r].recv_off[i] * es, B(r) + g[r].recv_off[i] * es,
               SNAP(q) + g[q].send_off[i] * es, g[r].recv_cnt[i]);
      }
    }
    /* 2. up the chain of blocks, smallest first: fold the smaller block's scattered pieces.
     * Blocks sit at decreasing rank offsets as they grow, so walk block offsets downwards. */
    for (int r = P - 1; r >= 0; r = (int)g[r].off - 1) {
      const uint32_t bo = g[r].off, bsz = g[r].size;
      if (!g[r].smaller) continue;
      for (uint32_t l = bo; l < bo + bsz; l++) {
        const hd_rank* L = &g[l];
        const size_t want = L->recv_cnt[L->steps - 1];
        if (!want) continue;
        const int s = (int)(bo + bsz + L->rib % L->smaller);
        const hd_rank* S = &g[s];
        const size_t total = S->steps ? S->recv_cnt[S->steps - 1] : n;
        const size_t soff = S->steps ? S->recv_off[S->steps - 1] : 0;
        const uint32_t k = L->size / S->size, ord = hd_rev(S->rib, S->steps) * k;
        int found = 0;
        for (uint32_t i = 0; i < k; i++) {
          if (S->sc_larger * i >= total) break;
          if (S->off - L->size + hd_rev(ord + i, L->steps) != l) continue;
          const size_t len = total - S->sc_larger * i < S->sc_larger ? total - S->sc_larger * i
                                                                      : S->sc_larger;
          if (len != want) { rc = 4; goto out; }
          unsigned char* dst = B(l) + L->recv_off[L->steps - 1] * es;
          orc_op(op, dtype, dst, dst, B(s) + (soff + i * S->sc_larger) * es, want);
          found = 1;
        }
        if (!found) { rc = 5; goto out; }
      }
    }
    /* 3. down the chain, largest first: the smaller block copies the finished pieces. */
    for (int r = 0; r < P; r += (int)g[r].size) {
      if (!g[r].larger) continue;
      const uint32_t bo = g[r].off, bsz = g[r].size;
      for (uint32_t s = bo; s < bo + bsz; s++) {
        const hd_rank* S = &g[s];
        const size_t total = S->steps ? S->recv_cnt[S->steps - 1] : n;
        const size_t soff = S->steps ? S->recv_off[S->steps - 1] : 0;
        if (!total) continue;
        const uint32_t k = S->larger / S->size, ord = hd_rev(S->rib, S->steps) * k;
        for (uint32_t i = 0; i < k; i++) {
          if (S->sc_larger * i >= total) break;
          const int l = (int)(S->off - S->larger + hd_rev(ord + i, hd_log2(S->larger)));
          const hd_rank* L = &g[l];
          const size_t len = total - S->sc_larger * i < S->sc_larger ? total - S->sc_larger * i
                                                                      : S->sc_larger;
          if (L->off + L->size + L->rib % L->smaller != s || L->recv_cnt[L->steps - 1] != len) {
            rc = 6;
            goto out;
          }
          memcpy(B(s) + (soff + i * S->sc_larger) * es, B(l) + L->recv_off[L->steps - 1] * es,
                 len * es);
        }
      }
    }
    /* 4. allgather inside every block, last step first */
    for (int i = (int)max_steps - 1; i >= 0; i--) {
      for (int r = 0; r < P; r++) memcpy(SNAP(r), B(r), n * es);
      for (int r = 0; r < P; r++) {
        if (g[r].steps <= (uint32_t)i || !g[r].send_cnt[i]) continue;
        const int q = r ^ (1 << i);
        memcpy(B(r) + g[r].send_off[i] * es, SNAP(q) + g[q].recv_off[i] * es, g[r].send_cnt[i] * es);
      }
    }
  out:
#undef B
#undef SNAP
    free(g);
    free(snap);
  }
  if (!rc)
    for (int r = 0; r < P; r++)
      for (int i = 1; i < nptr; i++) memcpy(bufs[r * nptr + i], bufs[r * nptr], n * es);
  return rc;
}

/* ReductionFunction<T>::Function-shaped (x = x op y) entry points for host-runtime tests. */
void orc_isum_f32(void* x, const void* y, size_t n) { orc_op(OP_SUM, D_FLOAT32, x, x, y, n); }
void orc_isum_i32(void* x, const void* y, size_t n) { orc_op(OP_SUM, D_INT32, x, x, y, n); }
void orc_isum_f16(void* x, const void* y, size_t n) { orc_op(OP_SUM, D_FLOAT16, x, x, y, n); }

/* ---- new-style gloo::reduce (reduce.cc:21-262) ----
 * Segment geometry (reduce.cc:87-135) differs from the allreduce ring's: segmentBytes =
 * roundUp(min(ceil(B / 2P), maxSegmentSize rounded down to E), E), then numSegments =
 * roundUp(max(ceil(B / segmentBytes), 2P), P).  The reduce-scatter is the ring's (send to
 * rank-1, receive from rank+1, reduce(out + off, in + off, tmp)), so segment k's owner q = k / S
 * ends with x_q + (x_{q+1} + (... + x_{q-1})); rank q then sends its chunk to the root
 * (reduce.cc:229-261).  Only the root's output is defined; this restatement writes out[root]. */
void orc_reduce_plan(int P, size_t n, size_t esize, size_t max_segment, size_t* num_segments,
                     size_t* segment_bytes, size_t* segments_per_rank) {
  size_t total = n * esize;
  size_t max_seg_bytes = esize * (max_segment / esize);
  size_t half = (total + (size_t)P * 2 - 1) / ((size_t)P * 2);
  size_t sb = half < max_seg_bytes ? half : max_seg_bytes;
  if (sb % esize) sb += esize - sb % esize;
  size_t want = sb ? (total + sb - 1) / sb : 0;
  size_t ns = want > (size_t)P * 2 ? want : (size_t)P * 2;
  if (ns % (size_t)P) ns += (size_t)P - ns % (size_t)P;
  *num_segments = ns;
  *segment_bytes = sb;
  *segments_per_rank = ns / (size_t)P;
}

int orc_reduce(int P, int op, int dtype, size_t n, void** in, void** out, int root,
               size_t max_segment) {
  size_t es = orc_esize(dtype);
  if (!es || P < 1 || root < 0 || root >= P) return 1;
  if (n == 0) return 0;
  size_t bytes = n * es;
  if (P == 1) {
    if (in && in[0] != out[0]) memcpy(out[0], in[0], bytes);
    return 0;
  }
  size_t ns, sb, S;
  orc_reduce_plan(P, n, es, max_segment ? max_segment : (1u << 20), &ns, &sb, &S);
  if (!sb) return 1;
  unsigned char* acc = (unsigned char*)malloc(bytes + 1);
  unsigned char* tmp = (unsigned char*)malloc(sb + 1);
  if (!acc || !tmp) { free(acc); free(tmp); return 2; }
  for (size_t k = 0; k < ns; k++) {
    size_t off = k * sb;
    if (off >= bytes) break;
    size_t len = (bytes - off < sb) ? bytes - off : sb;
    size_t cnt = len / es;
    int q = (int)(k / S);
    const unsigned char* src = (const unsigned char*)(in ? in : out)[(q + P - 1) % P];
    memcpy(acc + off, src + off, len);
    for (int d = P - 2; d >= 0; d--) {
      int j = (q + d) % P;
      memcpy(tmp, (const unsigned char*)(in ? in : out)[j] + off, len);
      orc_op(op, dtype, tmp, tmp, acc + off, cnt);
      memcpy(acc + off, tmp, len);
    }
  }
  memcpy(out[root], acc, bytes);
  free(acc);
  free(tmp);
  return 0;
}
