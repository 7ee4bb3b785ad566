// knn_driver.cpp -- drop-in replacement for the reference program
// (/root/reference/knn_mpi.cpp main(), cpp:86-399) on MI355X GPUs.
//
// Same inputs, same outputs:
//   * config: the reference's constants (cpp:108-119) become flags with the
//     same names and defaults: --dim 784 --K 50 --N_train 60000
//     --N_test 10000 --N_val 10000 --class_cnt 10 --Euclidean_distance true
//     --Normalize true --Validation true --train_file mnist_train.csv
//     --validation_file mnist_validation.csv --test_file mnist_test.csv
//   * inputs: the same CSV formats (cpp:154-222, see csv.h)
//   * outputs: "accuracy = <cout default>" (cpp:348), Test_label.csv one
//     label per line (cpp:390-392), "Running time is <t> second" (cpp:398)
// Extra flags: --gpus N (default 1), --mode query|train (multi-GPU layout),
// --strict (exit 1 unless N_* divisible by --gpus, as MPI_Abort cpp:127-129),
// --threads T (CSV parsing threads), --output path, --timings (per-phase
// seconds on stderr; stdout stays the reference's).
// The timed region spans the same work as the reference (barrier to
// barrier: CSV parsing, distribution, normalisation, both passes, output).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "csv.h"
#include "knn_amd.h"

namespace {

struct Config {
  int dim = 784;
  int K = 50;
  long long N_train = 60000, N_test = 10000, N_val = 10000;
  int class_cnt = 10;
  bool Euclidean_distance = true, Normalize = true, Validation = true;
  std::string train_file = "mnist_train.csv";
  std::string validation_file = "mnist_validation.csv";
  std::string test_file = "mnist_test.csv";
  std::string output = "Test_label.csv";
  int gpus = 1;
  int mode = 0;
  bool strict = false;
  int threads = 0;
  bool timings = false;
};

bool parse_bool(const std::string& v) { return v == "true" || v == "1" || v == "yes"; }

void usage() {
  fprintf(stderr,
          "usage: knn_mpi_amd [--dim D] [--K K] [--N_train N] [--N_test N] [--N_val N]\n"
          "  [--class_cnt C] [--Euclidean_distance true|false] [--Normalize true|false]\n"
          "  [--Validation true|false] [--train_file F] [--validation_file F]\n"
          "  [--test_file F] [--output F] [--gpus G] [--mode query|train] [--strict]\n"
          "  [--threads T] [--timings]\n");
}

int parse_args(int argc, char** argv, Config& c) {
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if (a == "-h" || a == "--help") { usage(); exit(0); }
    if (a.rfind("--", 0) != 0) { usage(); return 1; }
    a = a.substr(2);
    std::string v;
    size_t eq = a.find('=');
    if (eq != std::string::npos) { v = a.substr(eq + 1); a = a.substr(0, eq); }
    else if (a == "strict") { c.strict = true; continue; }
    else if (a == "timings") { c.timings = true; continue; }
    else if (i + 1 < argc) v = argv[++i];
    else { usage(); return 1; }
    if (a == "dim") c.dim = atoi(v.c_str());
    else if (a == "K") c.K = atoi(v.c_str());
    else if (a == "N_train") c.N_train = atoll(v.c_str());
    else if (a == "N_test") c.N_test = atoll(v.c_str());
    else if (a == "N_val") c.N_val = atoll(v.c_str());
    else if (a == "class_cnt") c.class_cnt = atoi(v.c_str());
    else if (a == "Euclidean_distance") c.Euclidean_distance = parse_bool(v);
    else if (a == "Normalize") c.Normalize = parse_bool(v);
    else if (a == "Validation") c.Validation = parse_bool(v);
    else if (a == "train_file") c.train_file = v;
    else if (a == "validation_file") c.validation_file = v;
    else if (a == "test_file") c.test_file = v;
    else if (a == "output") c.output = v;
    else if (a == "gpus") c.gpus = atoi(v.c_str());
    else if (a == "mode") c.mode = (v == "train" || v == "1") ? 1 : 0;
    else if (a == "strict") c.strict = parse_bool(v);
    else if (a == "threads") c.threads = atoi(v.c_str());
    else { fprintf(stderr, "unknown flag --%s\n", a.c_str()); usage(); return 1; }
  }
  return 0;
}

[[noreturn]] void die(const std::string& msg) {
  fprintf(stderr, "knn_mpi_amd: %s\n", msg.c_str());
  exit(1);  // ≙ MPI_Abort(MPI_COMM_WORLD, 1)
}

void load(const std::string& path, int dim, bool with_label, int64_t rows, std::vector<double>& X,
          std::vector<int32_t>* lab, int threads) {
  X.assign((size_t)rows * dim, 0.0);
  if (lab) lab->assign((size_t)rows, 0);
  knnhost::CsvResult r =
      knnhost::read_csv(path, dim, with_label, rows, X.data(), lab ? lab->data() : nullptr, threads);
  if (!r.ok) die(r.error);
  const int64_t want = rows * (dim + (with_label ? 1 : 0));
  if (r.tokens != want)
    die(path + ": expected " + std::to_string(want) + " values, found " + std::to_string(r.tokens));
}

}  // namespace

int main(int argc, char** argv) {
  Config c;
  if (parse_args(argc, argv, c)) return 1;
  if (c.threads <= 0) c.threads = (int)std::max(1u, std::thread::hardware_concurrency());
  if (c.threads > 16) c.threads = 16;
  if (c.gpus < 1) die("--gpus must be >= 1");
  if (c.dim <= 0 || c.K < 0 || c.N_train <= 0 || c.N_test < 0 || c.N_val < 0 || c.class_cnt <= 0)
    die("bad configuration");
  if (c.strict && (c.N_train % c.gpus || c.N_test % c.gpus || (c.Validation && c.N_val % c.gpus)))
    die("N_train/N_test/N_val not divisible by the number of GPUs (--strict, cpp:127-129)");

  knn_group* g = nullptr;
  if (knn_group_create(&g, c.gpus, nullptr, c.mode)) die(knn_last_error());

  using clk = std::chrono::steady_clock;
  const auto start = clk::now();  // ≙ MPI_Barrier + MPI_Wtime, cpp:133-134
  auto mark = start;
  auto phase = [&](const char* name) {
    const auto now = clk::now();
    if (c.timings)
      fprintf(stderr, "[knn_mpi_amd] %-10s %.3f s\n", name,
              std::chrono::duration<double>(now - mark).count());
    mark = now;
  };

  std::vector<double> Xtr, Xte, Xva;
  std::vector<int32_t> Ltr, Lva;
  load(c.train_file, c.dim, true, c.N_train, Xtr, &Ltr, c.threads);
  load(c.test_file, c.dim, false, c.N_test, Xte, nullptr, c.threads);
  if (c.Validation) load(c.validation_file, c.dim, true, c.N_val, Xva, &Lva, c.threads);
  phase("csv");

  if (c.Normalize) {  // cpp:229-306 on the GPUs: sharded min/max + RCCL all-reduce + apply
    std::vector<double*> sets{Xtr.data(), Xte.data()};
    std::vector<int64_t> rows{c.N_train, c.N_test};
    if (c.Validation) { sets.push_back(Xva.data()); rows.push_back(c.N_val); }
    if (knn_group_normalize(g, sets.data(), rows.data(), (int32_t)sets.size(), c.dim))
      die(knn_last_error());
  }
  phase("normalize");

  if (knn_group_set_train(g, Xtr.data(), Ltr.data(), c.N_train, c.dim, c.class_cnt))
    die(knn_last_error());
  phase("set_train");
  const int metric = c.Euclidean_distance ? KNN_METRIC_L2 : KNN_METRIC_L1;

  if (c.Validation) {  // cpp:308-349
    std::vector<int32_t> pred(c.N_val);
    if (c.N_val > 0 &&
        knn_group_classify(g, Xva.data(), c.N_val, c.K, metric, pred.data(), nullptr, nullptr, nullptr))
      die(knn_last_error());
    double acc = 0;  // acc_calc, cpp:69-84
    for (long long i = 0; i < c.N_val; i++)
      if (Lva[i] == pred[i]) acc++;
    acc /= c.N_val;
    std::cout << "accuracy = " << acc << std::endl;
    phase("validation");
  }

  std::vector<int32_t> test_lab(c.N_test);  // cpp:352-393
  if (c.N_test > 0 &&
      knn_group_classify(g, Xte.data(), c.N_test, c.K, metric, test_lab.data(), nullptr, nullptr, nullptr))
    die(knn_last_error());
  phase("test");
  {
    // one label per line (cpp:390-392; '\n' without a flush per line)
    std::ofstream outfile(c.output);
    for (long long i = 0; i < c.N_test; i++) outfile << test_lab[i] << '\n';
  }
  phase("output");

  const auto finish = clk::now();  // cpp:395-396
  knn_group_destroy(g);
  std::cout << "Running time is " << std::chrono::duration<double>(finish - start).count()
            << " second" << std::endl;
  return 0;
}
