// matrixfact_split — SGD matrix factorization over the petuum_ps App API, the C1 workload
// (BASELINE.json configs[0]: apps/matrixfact/src/matrixfact_split.cpp of the reference).
// Same algorithm and table layout: L (N x K) is thread-local, R (M x K, table 1,
// DenseRow<float>) and the loss table (table 2, 6 columns) live in the parameter server;
// each nonzero X(i,j) reads R(:,j) through Get and sends its update with DenseBatchInc;
// every worker clocks num_clocks_per_iter times per sweep.  Written against
// include/petuum_ps_common only (no gflags/glog/boost): flags are "--name value".
//
//   matrixfact_split --datafile X --K 16 --num_worker_threads 2 --num_iterations 4 ...
//
// The data file is the data_split binary format (data_split.cpp:200-217), partition
// suffix ".<client_id>": size_t nnz, rows, cols; int rows[nnz]; int cols[nnz];
// float vals[nnz], nonzeros grouped by row.
//
// Built with -DMF_ADAREVISION this is matrixfact_adarevision
// (apps/matrixfact/src/matrixfact_adarevision.cpp): R's table registers
// AdaRevisionServerTableLogic as server_table_logic 1 with version_maintain and
// no_oplog_replay (run_matrixfact_adarevision.sh:113-116), R's rows are initialised by the
// logic on the server, L steps with per-coordinate AdaGrad and R receives raw gradients.
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include <petuum_ps_common/include/petuum_ps.hpp>
#ifdef MF_ADAREVISION
#include <petuum_ps/server/adarevision_server_table_logic.hpp>
#endif

namespace {

std::map<std::string, std::string> g_flags;

double flag_d(const char *n, double dflt) {
  auto it = g_flags.find(n);
  return it == g_flags.end() ? dflt : std::atof(it->second.c_str());
}
int flag_i(const char *n, int dflt) { return (int)flag_d(n, dflt); }
bool flag_b(const char *n, bool dflt) {
  auto it = g_flags.find(n);
  return it == g_flags.end() ? dflt : (it->second == "true" || it->second == "1");
}
std::string flag_s(const char *n, const std::string &dflt) {
  auto it = g_flags.find(n);
  return it == g_flags.end() ? dflt : it->second;
}

[[noreturn]] void fail(const std::string &m) {
  std::fprintf(stderr, "matrixfact_split: %s\n", m.c_str());
  std::exit(1);
}

int K, num_iterations, num_clocks_per_iter, num_clocks_per_eval, num_worker_threads, num_clients, client_id;
double init_step_size, step_dec, lambda_;
bool use_step_dec;
int nnz_per_row, nnz_per_col;

size_t X_num_rows, X_num_cols;
std::vector<int> X_row, X_col;
std::vector<float> X_val;
std::vector<int64_t> X_partition_starts;

const int kLossClock = 0, kLossComputeTime = 1, kLossL2 = 2, kLossL2Reg = 3, kLossComputeEvalTime = 4, kLossIter = 5;

void ReadBinaryMatrix(const std::string &filename, int partition_id) {
  const std::string f = filename + "." + std::to_string(partition_id);
  FILE *in = std::fopen(f.c_str(), "rb");
  if (!in) fail("failed to read " + f);
  size_t nnz = 0, rows = 0, cols = 0;
  if (std::fread(&nnz, sizeof(size_t), 1, in) != 1 || std::fread(&rows, sizeof(size_t), 1, in) != 1 ||
      std::fread(&cols, sizeof(size_t), 1, in) != 1)
    fail("short header in " + f);
  X_row.resize(nnz);
  X_col.resize(nnz);
  X_val.resize(nnz);
  if (std::fread(X_row.data(), sizeof(int), nnz, in) != nnz || std::fread(X_col.data(), sizeof(int), nnz, in) != nnz ||
      std::fread(X_val.data(), sizeof(float), nnz, in) != nnz)
    fail("short body in " + f);
  std::fclose(in);
  X_num_rows = rows;
  X_num_cols = cols;
}

// Split the nonzeros into contiguous ranges that do not cut a row (matrixfact_split.cpp:99-126).
void PartitionWorkLoad(int workers) {
  const int64_t nnz = (int64_t)X_val.size();
  const int64_t per = nnz / workers;
  X_partition_starts.assign(workers, 0);
  int64_t start = 0;
  for (int w = 0; w < workers; ++w) {
    X_partition_starts[w] = start;
    if (w == workers - 1) break;
    int64_t end = start + per;
    const int end_row = X_row[end];
    while (end < nnz && X_row[end] == end_row) ++end;
    if (end >= nnz) fail("empty bin " + std::to_string(w));
    start = end;
  }
}

class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> l(m_);
    const int64_t gen = gen_;
    if (++arrived_ == n_) {
      arrived_ = 0;
      ++gen_;
      cv_.notify_all();
      return;
    }
    cv_.wait(l, [&] { return gen_ != gen; });
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, arrived_ = 0;
  int64_t gen_ = 0;
};

void ReadR(petuum::Table<float> &R, int j, std::vector<float> *cache) {
  petuum::RowAccessor acc;
  const auto &row = R.Get<petuum::DenseRow<float>>(j, &acc);
  row.CopyToVector(cache);
}

#ifdef MF_ADAREVISION
// matrixfact_adarevision.cpp:194-276: L steps by AdaGrad (history starts at 1), R gets the
// raw gradient and the server's AdaRevision logic turns it into a step
void SgdElement(int64_t a, float step_size, std::vector<std::vector<float>> &L, std::vector<std::vector<float>> &Lh,
                size_t L_off, petuum::Table<float> &R, std::vector<float> *Rj_cache) {
  const int i = X_row[a], j = X_col[a];
  const float Xij = X_val[a];
  ReadR(R, j, Rj_cache);
  auto &Rj = *Rj_cache;
  auto &Li = L[i - L_off];
  auto &Lhi = Lh[i - L_off];
  float LiRj = 0.0f;
  for (int k = 0; k < K; ++k) LiRj += Li[k] * Rj[k];
  petuum::DenseUpdateBatch<float> upd(0, K);
  const float grad_coeff = -(Xij - LiRj);
  const float reg = (float)lambda_;
  for (int k = 0; k < K; ++k) upd[k] = 0.f;
  for (int k = 0; k < K; ++k) {
    const float Lg = 2 * (grad_coeff * Rj[k] + reg / float(nnz_per_row) * Li[k]);
    const float Rg = 2 * (grad_coeff * Li[k] + reg / float(nnz_per_col) * Rj[k]);
    Lhi[k] += Lg * Lg;
    Li[k] -= step_size / std::sqrt(Lhi[k]) * Lg;
    upd[k] += Rg;
  }
  R.DenseBatchInc(j, upd);
}
#else

void SgdElement(int64_t a, float step_size, std::vector<std::vector<float>> &L, size_t L_off,
                petuum::Table<float> &R, std::vector<float> *Rj_cache) {
  const int i = X_row[a], j = X_col[a];
  const float Xij = X_val[a];
  ReadR(R, j, Rj_cache);
  auto &Rj = *Rj_cache;
  auto &Li = L[i - L_off];
  float LiRj = 0.0f;
  for (int k = 0; k < K; ++k) LiRj += Li[k] * Rj[k];
  petuum::DenseUpdateBatch<float> upd(0, K);
  const float grad_coeff = -2 * (Xij - LiRj);
  const float reg = (float)lambda_ * 2;
  for (int k = 0; k < K; ++k) {
    float g = grad_coeff * Rj[k] + reg / float(nnz_per_row) * Li[k];
    Li[k] += -g * step_size;
    g = grad_coeff * Li[k] + reg / float(nnz_per_col) * Rj[k];
    upd[k] = -g * step_size;
  }
  R.DenseBatchInc(j, upd);
}
#endif

void InitMF(std::vector<std::vector<float>> &L, petuum::Table<float> &R, int col_begin, int col_end) {
#ifdef MF_ADAREVISION
  // matrixfact_adarevision.cpp:278-291: L only (seed 12345); R's rows are drawn by the
  // server logic when they are created (ServerRowCreated)
  std::mt19937 gen(12345);
  std::normal_distribution<float> dist(0, 0.1);
  for (auto &row : L)
    for (int k = 0; k < K; ++k) row[k] = dist(gen);
  (void)R;
  (void)col_begin;
  (void)col_end;
#else
  std::mt19937 gen(1234);
  std::normal_distribution<float> dist(0, 0.1);
  for (auto &row : L)
    for (int k = 0; k < K; ++k) row[k] = dist(gen);
  for (int j = col_begin; j < col_end; ++j) {
    petuum::DenseUpdateBatch<float> u(0, K);
    for (int k = 0; k < K; ++k) u[k] = dist(gen);
    R.DenseBatchInc(j, u);
  }
#endif
}

void RecordLoss(int eval, int iter, int clock, std::vector<std::vector<float>> &L, size_t L_off,
                petuum::Table<float> &R, petuum::Table<float> &loss, int col_begin, int col_end,
                int gwid, int64_t eb, int64_t ee, std::vector<float> *Rj_cache) {
  float sq = 0.f;
  for (int64_t a = eb; a < ee; ++a) {
    ReadR(R, X_col[a], Rj_cache);
    auto &Li = L[X_row[a] - L_off];
    float LiRj = 0.f;
    for (int k = 0; k < K; ++k) LiRj += Li[k] * (*Rj_cache)[k];
    sq += std::pow(X_val[a] - LiRj, 2);
  }
  loss.Inc(eval, kLossL2, sq);
  if (gwid == 0) {
    loss.Inc(eval, kLossClock, (float)clock);
    loss.Inc(eval, kLossIter, (float)iter);
  }
  float reg = 0.f;
  for (auto &Li : L)
    for (int k = 0; k < K; ++k) reg += Li[k] * Li[k];
  for (int c = col_begin; c < col_end; ++c) {
    ReadR(R, c, Rj_cache);
    for (int k = 0; k < K; ++k) reg += (*Rj_cache)[k] * (*Rj_cache)[k];
  }
  reg *= (float)lambda_;
  loss.Inc(eval, kLossL2Reg, reg + sq);
}

void SolveMF(int tid, Barrier *process_barrier) {
  petuum::PSTableGroup::RegisterThread();
  petuum::Table<float> R = petuum::PSTableGroup::GetTableOrDie<float>(1);
  petuum::Table<float> loss = petuum::PSTableGroup::GetTableOrDie<float>(2);

  // InitLTable: this thread's rows [first row of its range, last row]
  const int row_st = X_row[X_partition_starts[tid]];
  const int row_end = tid == (int)X_partition_starts.size() - 1 ? X_row.back()
                                                                 : X_row[X_partition_starts[tid + 1] - 1];
  std::vector<std::vector<float>> L(row_end - row_st + 1, std::vector<float>(K, 0.f));
#ifdef MF_ADAREVISION
  std::vector<std::vector<float>> Lh(L.size(), std::vector<float>(K, 1.f));   // InitLTable :186
#endif
  const size_t L_off = row_st;

  const int total_workers = num_clients * num_worker_threads;
  const int gwid = client_id * num_worker_threads + tid;
  const int cols_per = (int)X_num_cols / total_workers;
  const int col_begin = gwid * cols_per;
  const int col_end = gwid == total_workers - 1 ? (int)X_num_cols : col_begin + cols_per;
  std::vector<float> Rj_cache(K);

  InitMF(L, R, col_begin, col_end);
  petuum::PSTableGroup::GlobalBarrier();

  const int64_t eb = X_partition_starts[tid];
  const int64_t ee = tid == num_worker_threads - 1 ? (int64_t)X_row.size() : X_partition_starts[tid + 1];
  const int64_t work_per_clock = (ee - eb) / num_clocks_per_iter;
  if (work_per_clock <= 0) fail("work_per_clock < 1: reduce num_clocks_per_iter");

  if (tid == 0) {   // bootstrap: fetch every R row this process touches
    std::set<int32_t> rows(X_col.begin(), X_col.end());
    for (int r : rows) R.GetAsyncForced(r);
    R.WaitPendingAsyncGet();
  }
  process_barrier->wait();
  petuum::PSTableGroup::GlobalBarrier();

  petuum::HighResolutionTimer total_timer;
  double total_eval = 0.;
  int clock = 0, eval = 0;
  for (int iter = 0; iter < num_iterations; ++iter) {
#ifdef MF_ADAREVISION
    const float step = (float)init_step_size;   // :507
#else
    const float step = use_step_dec ? (float)(init_step_size * std::pow(step_dec, iter))
                                    : (float)(init_step_size * std::pow(100.0 + iter, -0.5));
#endif
    int64_t counter = 0;
    for (int64_t a = eb; a < ee; ++a) {
#ifdef MF_ADAREVISION
      SgdElement(a, step, L, Lh, L_off, R, &Rj_cache);
#else
      SgdElement(a, step, L, L_off, R, &Rj_cache);
#endif
      ++counter;
      if ((counter % work_per_clock == 0 && clock < (iter + 1) * num_clocks_per_iter - 1) || counter == ee - eb) {
        petuum::PSTableGroup::Clock();
        ++clock;
        {
          petuum::RowAccessor acc;   // a fake Get to avoid the initial block time
          R.Get(X_col[a], &acc);
        }
        if (clock % num_clocks_per_eval == 0) {
          petuum::HighResolutionTimer et;
          RecordLoss(eval, iter + 1, clock, L, L_off, R, loss, col_begin, col_end, gwid, eb, ee, &Rj_cache);
          const double cost = et.elapsed();
          total_eval += cost;
          if (gwid == 0 && eval > 0) {
            const double total = total_timer.elapsed();
            loss.Inc(eval, kLossComputeTime, (float)(total - total_eval));
            loss.Inc(eval, kLossComputeEvalTime, (float)total);
          }
          ++eval;
        }
      }
    }
    if (clock != (iter + 1) * num_clocks_per_iter) fail("clock count");
  }
  petuum::PSTableGroup::GlobalBarrier();

  if (gwid == 0) {
    std::printf("Iter Clock Compute-Time Compute-Eval-Time L2_loss L2_reg_loss\n");
    for (int c = 0; c < eval; ++c) {
      petuum::RowAccessor acc;
      loss.Get(c, &acc);
      const auto &row = acc.Get<petuum::DenseRow<float>>();
      std::printf("LOSS %g %g %g %g %.9g %.9g\n", row[kLossIter], row[kLossClock], row[kLossComputeTime],
                  row[kLossComputeEvalTime], row[kLossL2], row[kLossL2Reg]);
    }
    std::fflush(stdout);
  }
  petuum::PSTableGroup::DeregisterThread();
}

}  // namespace

int main(int argc, char **argv) {
  for (int i = 1; i + 1 < argc; i += 2) {
    if (std::strncmp(argv[i], "--", 2)) fail(std::string("bad flag ") + argv[i]);
    g_flags[argv[i] + 2] = argv[i + 1];
  }
  K = flag_i("K", 100);
  num_iterations = flag_i("num_iterations", 100);
  num_clocks_per_iter = flag_i("num_clocks_per_iter", 1);
  num_clocks_per_eval = flag_i("num_clocks_per_eval", 1);
  num_worker_threads = flag_i("num_worker_threads", 1);
  num_clients = flag_i("num_clients", 1);
  client_id = flag_i("client_id", 0);
  init_step_size = flag_d("init_step_size", 0.5);
  step_dec = flag_d("step_dec", 0.9);
  use_step_dec = flag_b("use_step_dec", false);
  lambda_ = flag_d("lambda", 0.001);
  nnz_per_row = flag_i("nnz_per_row", 1);
  nnz_per_col = flag_i("nnz_per_col", 1);
  const int staleness = flag_i("table_staleness", 0);

  petuum::TableGroupConfig tg;
  petuum::InitTableGroupConfig(&tg, 2);
  tg.num_comm_channels_per_client = flag_i("num_comm_channels_per_client", 1);
  tg.num_total_clients = num_clients;
  tg.client_id = client_id;
  tg.num_local_app_threads = num_worker_threads + 1;
#ifdef MF_ADAREVISION
  // matrixfact_adarevision.cpp:633-635; its flag (DECLARE_double(init_step_size)) is the logic's
  FLAGS_init_step_size = init_step_size;
  petuum::ClassRegistry<petuum::AbstractServerTableLogic>::GetRegistry().AddCreator(
      1, petuum::CreateObj<petuum::AbstractServerTableLogic, petuum::AdaRevisionServerTableLogic>);
#endif
  petuum::PSTableGroup::RegisterRow<petuum::DenseRow<float>>(0);
  petuum::PSTableGroup::RegisterRow<petuum::DenseRow<int64_t>>(1);
  petuum::PSTableGroup::Init(tg, false);   // the init thread does not access tables

  ReadBinaryMatrix(flag_s("datafile", ""), client_id);
  PartitionWorkLoad(num_worker_threads);

  petuum::ClientTableConfig tc;
  petuum::InitTableConfig(&tc);
  tc.table_info.table_staleness = staleness;
  tc.table_info.server_push_row_upper_bound = flag_i("server_push_row_upper_bound", 100);
  tc.table_info.row_capacity = K;
  tc.table_info.dense_row_oplog_capacity = K;
  tc.table_info.row_oplog_type = flag_i("row_oplog_type", 0);
  tc.table_info.oplog_dense_serialized = flag_b("oplog_dense_serialized", true);
  tc.no_oplog_replay = flag_b("no_oplog_replay", false);
  tc.process_cache_capacity = (size_t)flag_i("M_cache_size", (int)X_num_cols);
  tc.oplog_capacity = tc.process_cache_capacity;
#ifdef MF_ADAREVISION
  // run_matrixfact_adarevision.sh:113-116
  tc.table_info.server_table_logic = flag_i("server_table_logic", 1);
  tc.table_info.version_maintain = flag_b("version_maintain", true);
  tc.no_oplog_replay = flag_b("no_oplog_replay", true);
#endif
  petuum::PSTableGroup::CreateTable(1, tc);
  tc.table_info.server_table_logic = -1;
  tc.table_info.version_maintain = false;

  tc.table_info.oplog_dense_serialized = true;
  tc.no_oplog_replay = false;
  tc.oplog_type = petuum::Sparse;
  tc.process_storage_type = petuum::BoundedSparse;
  tc.table_info.row_capacity = 6;
  tc.table_info.dense_row_oplog_capacity = 6;
  tc.table_info.row_oplog_type = 0;
  tc.process_cache_capacity = 100;
  tc.oplog_capacity = 100;
  petuum::PSTableGroup::CreateTable(2, tc);
  petuum::PSTableGroup::CreateTableDone();

  std::vector<std::thread> threads;
  Barrier barrier(num_worker_threads);
  for (int t = 0; t < num_worker_threads; ++t) threads.emplace_back(SolveMF, t, &barrier);
  for (auto &th : threads) th.join();
  petuum::PSTableGroup::ShutDown();
  return 0;
}
