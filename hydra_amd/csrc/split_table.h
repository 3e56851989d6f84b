// split_table.h -- the two-rail split of bew_allreduce_a (APipeAllreduceOptions::
// calculateElements_AA / _AG, gloo/gloo/pipeallreduce-a.h:137-376), shared by the host runtime
// (apipe_allreduce over two TCP contexts) and the device library (hydra_apipe_allreduce over
// two RCCL communicators).  e2 = w*(n - n mod ce)/ce elements go to rail 2, e1 = n - e2 to rail 1.
#pragma once

#include <cstddef>

namespace hydra {

inline void split_elements(int table, int P, size_t n, size_t* e1, size_t* e2) {
  int ce = 1, w = 1;
  if (table == 0) {  // calculateElements_AA (pipeallreduce-a.h:296-376)
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
  } else {  // calculateElements_AG (pipeallreduce-a.h:137-294)
    struct Band { size_t lo, hi; int w; };  // lo < n < hi  -> w_2 = w (cout_ele 100)
    if (P == 2) {
      ce = 100;
      static const Band b[] = {{524288, 1048577, 75}, {1048576, 2097153, 74},
                               {2097152, 4194305, 72}, {4194304, 8388609, 69},
                               {8388608, 16777217, 67}, {16777216, 33554433, 65},
                               {33554432, 67108865, 65}};
      if (n < 524289) { ce = 1; w = 1; }
      else {
        w = 60;
        for (const auto& x : b) if (x.lo < n && n < x.hi) { w = x.w; break; }
      }
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
    } else if (P == 4 || P == 6) {
      ce = 100;
      static const Band b4[] = {{828343, 1048577, 81}, {1048576, 2097153, 73},
                                {2097152, 4194305, 70}, {4194304, 8388609, 67},
                                {8388608, 16777217, 65}, {16777216, 33554433, 65},
                                {33554432, 67108865, 66}};
      static const Band b6[] = {{1048576, 2097153, 73}, {2097152, 4194305, 70},
                                {4194304, 8388609, 66}, {8388608, 16777217, 66},
                                {16777216, 33554433, 64}, {33554432, 67108865, 66}};
      const size_t small = P == 4 ? 828344 : 1048577;
      if (n < small) { ce = 1; w = 1; }
      else {
        ce = 2;
        w = 1;
        const Band* b = P == 4 ? b4 : b6;
        const size_t nb = P == 4 ? 7 : 6;
        for (size_t k = 0; k < nb; k++)
          if (b[k].lo < n && n < b[k].hi) { ce = 100; w = b[k].w; break; }
      }
    } else {
      if (n < 6145) { ce = 1; w = 0; } else { ce = 1; w = 1; }
    }
  }
  const int mode = (int)(n % (size_t)ce);
  *e2 = mode == 0 ? (size_t)w * n / (size_t)ce : (size_t)w * (n - (size_t)mode) / (size_t)ce;
  *e1 = n - *e2;
}

}  // namespace hydra
