// mlr_sgd — multiclass logistic regression by minibatch SGD over the petuum_ps App API,
// shaped like the reference's apps/mlr (mlr_main.cpp:70-108, mlr_sgd_solver.cpp:66-95):
//
//   W table     DenseRow<float> (row type 0), one row per label, feature_dim columns;
//               every refresh is one DenseBatchInc(label, w_delta[label]) of feature_dim
//               values, then every label row read back with Get (RefreshParamsDense)
//   loss table  DenseRow<float>, one row per evaluation {iter, loss, accuracy}
//
// with the reference's run_lr_synth.sh settings (row_oplog_type 0, --oplog_dense_serialized).
// Written against include/petuum_ps_common only (no gflags/glog/boost): flags are
// "--name value".  Data: a synthetic, linearly separable-ish multiclass set (--seed), or a
// libsvm file with its .meta (--train_file; the reference's ReadDataLabelLibSVM input, e.g.
// apps/mlr/datasets/covtype.scale.train.small: feature_dim 54, 7 labels, one-based features
// and labels), split evenly over the worker threads.
//
//   mlr_sgd --num_labels 8 --feature_dim 512 --num_train 4000 --num_worker_threads 2
//   mlr_sgd --train_file covtype.scale.train.small --num_worker_threads 2
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <petuum_ps_common/include/petuum_ps.hpp>

namespace {

std::map<std::string, std::string> g_flags;
double flag_d(const char *n, double dflt) {
  auto it = g_flags.find(n);
  return it == g_flags.end() ? dflt : std::atof(it->second.c_str());
}
int flag_i(const char *n, int dflt) { return (int)flag_d(n, dflt); }

[[noreturn]] void fail(const std::string &m) {
  std::fprintf(stderr, "mlr_sgd: %s\n", m.c_str());
  std::exit(1);
}

const int32_t kWTable = 0, kLossTable = 1, kDenseRowFloatTypeID = 0;
int num_labels, feature_dim, num_train, num_threads, num_epochs, batch_size;
double learning_rate, decay;

std::vector<std::vector<float>> X;
std::vector<int32_t> Y;

void MakeData(uint32_t seed) {
  std::mt19937 g(seed);
  std::normal_distribution<float> n01(0.f, 1.f);
  std::vector<std::vector<float>> centers(num_labels, std::vector<float>(feature_dim));
  for (auto &c : centers)
    for (auto &x : c) x = n01(g);
  X.assign(num_train, std::vector<float>(feature_dim));
  Y.resize(num_train);
  for (int i = 0; i < num_train; ++i) {
    Y[i] = (int32_t)(g() % (uint32_t)num_labels);
    for (int j = 0; j < feature_dim; ++j) X[i][j] = 0.25f * centers[Y[i]][j] + n01(g);
  }
}

// The reference's MetafileReader keys (ml/util/metafile_reader.cpp: "key: value" lines).
std::map<std::string, std::string> ReadMeta(const std::string &path) {
  std::ifstream f(path);
  if (!f) fail("cannot open " + path);
  std::map<std::string, std::string> m;
  std::string line;
  while (std::getline(f, line)) {
    const size_t c = line.find(':');
    if (c == std::string::npos) continue;
    std::string v = line.substr(c + 1);
    v.erase(0, v.find_first_not_of(" \t"));
    m[line.substr(0, c)] = v;
  }
  return m;
}

// libsvm rows "label idx:val ..." (ReadDataLabelLibSVM, ml/util/data_loading.cpp): features
// and labels shifted to zero-based when the meta file says they are one-based.
void ReadLibSVM(const std::string &path, const std::string &meta_path) {
  auto meta = ReadMeta(meta_path);
  auto need = [&](const char *k) {
    auto it = meta.find(k);
    if (it == meta.end()) fail(meta_path + " has no " + k);
    return std::atoi(it->second.c_str());
  };
  feature_dim = need("feature_dim");
  num_labels = need("num_labels");
  const int f1 = need("feature_one_based"), l1 = need("label_one_based");
  if (meta.count("format") && meta["format"] != "libsvm") fail("format " + meta["format"] + " is not libsvm");
  std::ifstream f(path);
  if (!f) fail("cannot open " + path);
  X.clear();
  Y.clear();
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream in(line);
    int label;
    if (!(in >> label)) continue;
    std::vector<float> x(feature_dim, 0.f);
    std::string tok;
    while (in >> tok) {
      const size_t c = tok.find(':');
      if (c == std::string::npos) fail("bad feature " + tok);
      const int j = std::atoi(tok.substr(0, c).c_str()) - f1;
      if (j < 0 || j >= feature_dim) fail("feature index out of range: " + tok);
      x[j] = std::strtof(tok.c_str() + c + 1, nullptr);
    }
    label -= l1;
    if (label < 0 || label >= num_labels) fail("label out of range in " + line);
    X.push_back(std::move(x));
    Y.push_back(label);
  }
  num_train = (int)X.size();
  if (!num_train) fail(path + " holds no rows");
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

// softmax(W x) in place of logits
void Predict(const std::vector<std::vector<float>> &W, const std::vector<float> &x, std::vector<float> *p) {
  float mx = -1e30f;
  for (int k = 0; k < num_labels; ++k) {
    float z = 0.f;
    for (int j = 0; j < feature_dim; ++j) z += W[k][j] * x[j];
    (*p)[k] = z;
    mx = std::max(mx, z);
  }
  float s = 0.f;
  for (int k = 0; k < num_labels; ++k) s += ((*p)[k] = std::exp((*p)[k] - mx));
  for (int k = 0; k < num_labels; ++k) (*p)[k] /= s;
}

// RefreshParamsDense (mlr_sgd_solver.cpp:66-95): send every label's delta, zero it, read W
void Refresh(petuum::Table<float> &w_table, std::vector<std::vector<float>> &delta,
             std::vector<std::vector<float>> &W) {
  for (int k = 0; k < num_labels; ++k) {
    petuum::DenseUpdateBatch<float> upd(0, feature_dim);
    for (int j = 0; j < feature_dim; ++j) upd[j] = delta[k][j];
    w_table.DenseBatchInc(k, upd);
    std::fill(delta[k].begin(), delta[k].end(), 0.f);
  }
  for (int k = 0; k < num_labels; ++k) {
    petuum::RowAccessor acc;
    const auto &row = w_table.Get<petuum::DenseRow<float>>(k, &acc);
    row.CopyToVector(&W[k]);
  }
}

void Worker(int tid, Barrier *barrier) {
  petuum::PSTableGroup::RegisterThread();
  auto w_table = petuum::PSTableGroup::GetTableOrDie<float>(kWTable);
  auto loss_table = petuum::PSTableGroup::GetTableOrDie<float>(kLossTable);
  const int i0 = (int)((int64_t)num_train * tid / num_threads), i1 = (int)((int64_t)num_train * (tid + 1) / num_threads);
  std::vector<std::vector<float>> W(num_labels, std::vector<float>(feature_dim, 0.f)),
      delta(num_labels, std::vector<float>(feature_dim, 0.f));
  std::vector<float> p(num_labels);
  Refresh(w_table, delta, W);   // every row zero: fetches W
  barrier->wait();
  petuum::PSTableGroup::GlobalBarrier();
  int eval = 0;
  for (int ep = 0; ep < num_epochs; ++ep) {
    const float lr = (float)(learning_rate * std::pow(decay, ep));
    int in_batch = 0;
    for (int i = i0; i < i1; ++i) {
      Predict(W, X[i], &p);
      // gradient of the cross-entropy: (p_k - [k == y]) x
      for (int k = 0; k < num_labels; ++k) {
        const float g = p[k] - (k == Y[i] ? 1.f : 0.f);
        for (int j = 0; j < feature_dim; ++j) {
          const float d = -lr * g * X[i][j];
          delta[k][j] += d;
          W[k][j] += d;   // the worker's own view moves between refreshes
        }
      }
      if (++in_batch == batch_size || i + 1 == i1) {
        Refresh(w_table, delta, W);
        in_batch = 0;
      }
    }
    // evaluate on this thread's shard: mean loss and accuracy, summed over threads
    double loss = 0;
    int correct = 0;
    for (int i = i0; i < i1; ++i) {
      Predict(W, X[i], &p);
      loss += -std::log(std::max(p[Y[i]], 1e-30f));
      int best = 0;
      for (int k = 1; k < num_labels; ++k)
        if (p[k] > p[best]) best = k;
      correct += best == Y[i];
    }
    loss_table.Inc(eval, 1, (float)(loss / num_train));
    loss_table.Inc(eval, 2, (float)correct / (float)num_train);
    if (tid == 0) loss_table.Inc(eval, 0, (float)(ep + 1));
    ++eval;
    petuum::PSTableGroup::Clock();
  }
  petuum::PSTableGroup::GlobalBarrier();
  if (tid == 0) {
    for (int e = 0; e < eval; ++e) {
      petuum::RowAccessor acc;
      loss_table.Get(e, &acc);
      const auto &row = acc.Get<petuum::DenseRow<float>>();
      std::printf("LOSS %g %.9g %.6g\n", row[0], row[1], row[2]);
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
  num_labels = flag_i("num_labels", 8);
  feature_dim = flag_i("feature_dim", 512);
  num_train = flag_i("num_train", 4000);
  num_threads = flag_i("num_worker_threads", 2);
  num_epochs = flag_i("num_epochs", 4);
  batch_size = flag_i("batch_size", 100);
  learning_rate = flag_d("learning_rate", 0.05);
  decay = flag_d("decay_rate", 0.9);
  const int staleness = flag_i("table_staleness", 0);
  if (g_flags.count("train_file")) {
    const std::string tf = g_flags["train_file"];
    ReadLibSVM(tf, g_flags.count("meta") ? g_flags["meta"] : tf + ".meta");
    std::printf("DATA %d %d %d\n", num_train, feature_dim, num_labels);
  } else {
    MakeData((uint32_t)flag_i("seed", 1234));
  }

  petuum::TableGroupConfig tg;
  petuum::InitTableGroupConfig(&tg, 2);
  tg.num_comm_channels_per_client = flag_i("num_comm_channels_per_client", 1);
  tg.num_local_app_threads = num_threads + 1;
  petuum::PSTableGroup::RegisterRow<petuum::DenseRow<float>>(kDenseRowFloatTypeID);
  petuum::PSTableGroup::Init(tg, false);

  // mlr_main.cpp:80-108 (num_labels > 2: one row per label of feature_dim columns)
  petuum::ClientTableConfig tc;
  petuum::InitTableConfig(&tc);
  tc.table_info.table_staleness = staleness;
  tc.table_info.row_type = kDenseRowFloatTypeID;
  tc.table_info.row_capacity = feature_dim;
  tc.table_info.dense_row_oplog_capacity = feature_dim;
  tc.table_info.oplog_dense_serialized = true;
  tc.process_cache_capacity = num_labels;
  tc.oplog_capacity = num_labels;
  if (!petuum::PSTableGroup::CreateTable(kWTable, tc)) fail("W table");
  tc.process_storage_type = petuum::BoundedSparse;
  tc.table_info.row_capacity = 3;
  tc.table_info.dense_row_oplog_capacity = 3;
  tc.process_cache_capacity = 1000;
  tc.oplog_capacity = 1000;
  if (!petuum::PSTableGroup::CreateTable(kLossTable, tc)) fail("loss table");
  petuum::PSTableGroup::CreateTableDone();

  std::vector<std::thread> threads;
  Barrier barrier(num_threads);
  for (int t = 0; t < num_threads; ++t) threads.emplace_back(Worker, t, &barrier);
  for (auto &th : threads) th.join();
  petuum::PSTableGroup::ShutDown();
  return 0;
}
