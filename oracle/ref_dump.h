// ref_dump.h -- instrumentation helper force-included (-include) into the
// oracle/_ref build of /root/reference/knn_mpi.cpp by oracle/build_ref.py.
// TEST INFRASTRUCTURE ONLY.
//
// build_ref.py adds an `int idx;` field to the reference's record
// (cpp:20; it lands in the 4 padding bytes, sizeof stays 16, and std::sort's
// permutation only depends on `dis`, so Test_label.csv is unchanged), sets it
// in the fill loops (cpp:319/362) and calls KNN_DUMP right after each
// std::sort (cpp:323/366).  When KNN_DUMP_N is set in the environment, each
// rank appends "global_query_index idx:dis ..." lines with the first
// KNN_DUMP_N sorted records to dump_<tag>_<rank>.txt (dis printed %.17g, so
// it round-trips the double exactly).
#pragma once
#include <cstdio>
#include <cstdlib>

#define KNN_DUMP(arr, tag, gi)                                                   \
  do {                                                                           \
    static FILE* knn_f_ = 0;                                                     \
    static int knn_n_ = -1;                                                      \
    if (knn_n_ < 0) {                                                            \
      const char* e_ = getenv("KNN_DUMP_N");                                     \
      knn_n_ = e_ ? atoi(e_) : 0;                                                \
      if (knn_n_ > 0) {                                                          \
        char nm_[64];                                                            \
        snprintf(nm_, sizeof nm_, "dump_%s_%d.txt", tag, myid);                  \
        knn_f_ = fopen(nm_, "w");                                                \
      }                                                                          \
    }                                                                            \
    if (knn_f_) {                                                                \
      fprintf(knn_f_, "%d", (int)(gi));                                          \
      for (int t_ = 0; t_ < N_train && t_ < knn_n_; t_++)                        \
        fprintf(knn_f_, " %d:%.17g", (arr)[t_].idx, (arr)[t_].dis);              \
      fprintf(knn_f_, "\n");                                                     \
      fflush(knn_f_);                                                            \
    }                                                                            \
  } while (0)
