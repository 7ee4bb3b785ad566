// csv.h -- reader for the reference's CSV formats (cpp:154-222).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace knnhost {

// Semantics of the reference loaders, reproduced exactly:
//  * the file is split into lines on '\n' (std::getline); each line is split
//    on ',' like std::getline(stringstream, token, ','): every segment
//    followed by a comma is a token (possibly empty), the last segment only
//    if it is non-empty;
//  * ONE running token counter spans the whole file, so rows come from the
//    count, not from line breaks;
//  * with_label: token c with c % (dim+1) == 0 is label c/(dim+1) (atoi),
//    every other token goes to data[c - c/(dim+1) - 1] (atof);
//    without label: token c goes to data[c] (atof).
// Differences (the reference has UB there): tokens beyond rows*(dim[+1])
// are not written (the reference overflows the heap) and a missing file is
// an error (the reference leaves the buffers uninitialised).
// Parsing is multi-threaded: a counting pass fixes each chunk's first token
// index, then the chunks are converted in parallel.
struct CsvResult {
  int64_t tokens = 0;  // tokens found in the file
  bool ok = false;
  std::string error;
};

CsvResult read_csv(const std::string& path, int dim, bool with_label, int64_t rows,
                   double* data, int32_t* labels, int threads);

}  // namespace knnhost
