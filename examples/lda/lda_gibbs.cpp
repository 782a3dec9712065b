// lda_gibbs — collapsed Gibbs LDA over the petuum_ps App API, shaped like the reference's
// apps/lda (lda_main.cpp:58-128, lda_engine.cpp:45-160, fast_doc_sampler.cpp:150-174):
//
//   word-topic table  SortedVectorMapRow<int32> (row type 1), one row per word, K topics;
//                     every reassignment is one BatchInc(word, {old: -1, new: +1})
//   summary table     DenseRow<int32> (row type 2), one row of K topic totals (Inc per change)
//   llh table         DenseRow<double> (row type 3), one row per iteration {iter, llh, time}
//
// with the reference's table settings (row_oplog_type 0, --nooplog_dense_serialized:
// sparse-serialized records, run_lda.sh:82-83; SSPPush, staleness from the flag).  Written
// against include/petuum_ps_common only (no gflags/glog/boost): flags are "--name value".
// The corpus is synthetic and deterministic (--seed): documents drawn from planted topics,
// so the log-likelihood rises as the sampler recovers them.
//
//   lda_gibbs --num_docs 400 --vocab 2000 --num_topics 32 --doc_len 50 --num_worker_threads 2
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
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
  std::fprintf(stderr, "lda_gibbs: %s\n", m.c_str());
  std::exit(1);
}

const int32_t kWordTopicTable = 1, kSummaryTable = 2, kLLHTable = 3;
const int32_t kSortedVectorMapRowTypeID = 1, kDenseRowIntTypeID = 2, kDenseRowDoubleTypeID = 3;

int num_docs, vocab, K, doc_len, num_threads, num_iterations;
double alpha, beta;

struct Doc {
  std::vector<int32_t> words, topics;
};
std::vector<Doc> corpus;

// Planted topics: topic t favours a contiguous band of the vocabulary; a document mixes
// two or three of them.
void MakeCorpus(uint32_t seed) {
  std::mt19937 g(seed);
  const int T = std::max(2, K / 2);
  corpus.resize(num_docs);
  for (int d = 0; d < num_docs; ++d) {
    std::uniform_int_distribution<int> pick(0, T - 1), len(doc_len / 2, doc_len);
    const int mix[3] = {pick(g), pick(g), pick(g)};
    const int n = len(g);
    auto &doc = corpus[d];
    for (int i = 0; i < n; ++i) {
      const int t = mix[g() % 3];
      const int band = std::max(1, vocab / T);
      std::geometric_distribution<int> off(4.0 / band);
      const int w = (t * band + std::min(off(g), band - 1)) % vocab;
      doc.words.push_back(w);
      doc.topics.push_back((int)(g() % (uint32_t)K));
    }
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

void Worker(int tid, Barrier *barrier) {
  petuum::PSTableGroup::RegisterThread();
  auto wt = petuum::PSTableGroup::GetTableOrDie<int32_t>(kWordTopicTable);
  auto summary = petuum::PSTableGroup::GetTableOrDie<int32_t>(kSummaryTable);
  auto llh = petuum::PSTableGroup::GetTableOrDie<double>(kLLHTable);
  const int d0 = (int)((int64_t)num_docs * tid / num_threads), d1 = (int)((int64_t)num_docs * (tid + 1) / num_threads);

  // tally the initial assignments, batched per word (lda_engine.cpp:57-76)
  {
    petuum::UpdateBatch<int32_t> sum_upd;
    std::map<int32_t, petuum::UpdateBatch<int32_t>> word_upd;
    std::vector<int32_t> tally(K, 0);
    for (int d = d0; d < d1; ++d)
      for (size_t i = 0; i < corpus[d].words.size(); ++i) {
        word_upd[corpus[d].words[i]].Update(corpus[d].topics[i], 1);
        ++tally[corpus[d].topics[i]];
      }
    for (int k = 0; k < K; ++k)
      if (tally[k]) sum_upd.Update(k, tally[k]);
    summary.BatchInc(0, sum_upd);
    for (auto &kv : word_upd) wt.BatchInc(kv.first, kv.second);
  }
  petuum::PSTableGroup::GlobalBarrier();
  barrier->wait();

  std::mt19937 rng(1000 + tid);
  std::vector<double> p(K);
  std::vector<int32_t> nd(K);
  for (int iter = 0; iter < num_iterations; ++iter) {
    petuum::HighResolutionTimer timer;
    for (int d = d0; d < d1; ++d) {
      Doc &doc = corpus[d];
      std::fill(nd.begin(), nd.end(), 0);
      for (int32_t t : doc.topics) ++nd[t];
      for (size_t i = 0; i < doc.words.size(); ++i) {
        const int32_t w = doc.words[i], old = doc.topics[i];
        std::vector<int32_t> nk(K);
        {
          petuum::RowAccessor acc;
          const auto &srow = summary.Get<petuum::DenseRow<int32_t>>(0, &acc);
          for (int k = 0; k < K; ++k) nk[k] = srow[k];
        }
        std::vector<int32_t> nw(K, 0);
        {
          petuum::RowAccessor acc;
          const auto &wrow = wt.Get<petuum::SortedVectorMapRow<int32_t>>(w, &acc);
          std::vector<petuum::Entry<int32_t>> ent;
          wrow.CopyToVector(&ent);
          for (auto &e : ent)
            if (e.first >= 0 && e.first < K) nw[e.first] = e.second;
        }
        --nd[old];
        double tot = 0;
        for (int k = 0; k < K; ++k) {
          const double nwk = std::max(0, nw[k] - (k == old ? 1 : 0));
          const double nkk = std::max(0, nk[k] - (k == old ? 1 : 0));
          p[k] = (nd[k] + alpha) * (nwk + beta) / (nkk + vocab * beta);
          tot += p[k];
        }
        double u = std::uniform_real_distribution<double>(0, tot)(rng);
        int32_t nt = K - 1;
        for (int k = 0; k < K; ++k) {
          u -= p[k];
          if (u <= 0) {
            nt = k;
            break;
          }
        }
        ++nd[nt];
        if (nt != old) {
          doc.topics[i] = nt;
          // fast_doc_sampler.cpp:164-174: the word's row gets -1 / +1 in one batch
          petuum::UpdateBatch<int32_t> upd(2);
          upd.UpdateSet(0, old, -1);
          upd.UpdateSet(1, nt, 1);
          wt.BatchInc(w, upd);
          summary.Inc(0, old, -1);
          summary.Inc(0, nt, 1);
        }
      }
    }
    // doc side of the complete log-likelihood (lda_stats.cpp ComputeOneDocLLH)
    double ll = 0;
    for (int d = d0; d < d1; ++d) {
      std::vector<int32_t> c(K, 0);
      for (int32_t t : corpus[d].topics) ++c[t];
      ll += std::lgamma(K * alpha) - std::lgamma(K * alpha + corpus[d].topics.size());
      for (int k = 0; k < K; ++k) ll += std::lgamma(c[k] + alpha) - std::lgamma(alpha);
    }
    llh.Inc(iter, 1, ll);
    if (tid == 0) {
      llh.Inc(iter, 0, (double)(iter + 1));
      llh.Inc(iter, 2, timer.elapsed());
    }
    petuum::PSTableGroup::Clock();
  }
  petuum::PSTableGroup::GlobalBarrier();
  if (tid == 0) {
    // word side, from the final word-topic and summary rows (ComputeWordLLH)
    double wl = 0;
    std::vector<int32_t> nk(K);
    {
      petuum::RowAccessor acc;
      const auto &srow = summary.Get<petuum::DenseRow<int32_t>>(0, &acc);
      for (int k = 0; k < K; ++k) nk[k] = srow[k];
    }
    for (int w = 0; w < vocab; ++w) {
      petuum::RowAccessor acc;
      const auto &wrow = wt.Get<petuum::SortedVectorMapRow<int32_t>>(w, &acc);
      std::vector<petuum::Entry<int32_t>> ent;
      wrow.CopyToVector(&ent);
      for (auto &e : ent) wl += std::lgamma(e.second + beta) - std::lgamma(beta);
    }
    for (int k = 0; k < K; ++k) wl += std::lgamma(vocab * beta) - std::lgamma(vocab * beta + nk[k]);
    int64_t tokens = 0;
    for (int k = 0; k < K; ++k) tokens += nk[k];
    for (int iter = 0; iter < num_iterations; ++iter) {
      petuum::RowAccessor acc;
      llh.Get(iter, &acc);
      const auto &row = acc.Get<petuum::DenseRow<double>>();
      std::printf("LLH %g %.12g %g\n", row[0], row[1], row[2]);
    }
    std::printf("WORDLLH %.12g TOKENS %lld\n", wl, (long long)tokens);
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
  num_docs = flag_i("num_docs", 400);
  vocab = flag_i("vocab", 2000);
  K = flag_i("num_topics", 32);
  doc_len = flag_i("doc_len", 50);
  num_threads = flag_i("num_worker_threads", 2);
  num_iterations = flag_i("num_iterations", 4);
  alpha = flag_d("alpha", 0.1);
  beta = flag_d("beta", 0.1);
  const int staleness = flag_i("table_staleness", 0);
  MakeCorpus((uint32_t)flag_i("seed", 1234));

  petuum::TableGroupConfig tg;
  petuum::InitTableGroupConfig(&tg, 3);
  tg.num_comm_channels_per_client = flag_i("num_comm_channels_per_client", 1);
  tg.num_local_app_threads = num_threads + 1;
  petuum::PSTableGroup::RegisterRow<petuum::SortedVectorMapRow<int32_t>>(kSortedVectorMapRowTypeID);
  petuum::PSTableGroup::RegisterRow<petuum::DenseRow<int32_t>>(kDenseRowIntTypeID);
  petuum::PSTableGroup::RegisterRow<petuum::DenseRow<double>>(kDenseRowDoubleTypeID);
  petuum::PSTableGroup::Init(tg, false);

  // lda_main.cpp:85-128, with run_lda.sh's --row_oplog_type 0 --nooplog_dense_serialized
  petuum::ClientTableConfig wt;
  petuum::InitTableConfig(&wt);
  wt.table_info.table_staleness = staleness;
  wt.table_info.oplog_dense_serialized = false;
  wt.table_info.row_capacity = K;
  wt.table_info.dense_row_oplog_capacity = K;
  wt.table_info.row_type = kSortedVectorMapRowTypeID;
  wt.process_cache_capacity = vocab;
  wt.oplog_capacity = vocab;
  wt.no_oplog_replay = true;
  if (!petuum::PSTableGroup::CreateTable(kWordTopicTable, wt)) fail("word-topic table");

  petuum::ClientTableConfig st;
  petuum::InitTableConfig(&st);
  st.table_info.table_staleness = staleness;
  st.table_info.oplog_dense_serialized = false;
  st.table_info.row_capacity = K;
  st.table_info.dense_row_oplog_capacity = K;
  st.table_info.row_type = kDenseRowIntTypeID;
  st.table_info.server_push_row_upper_bound = 1;
  st.process_storage_type = petuum::BoundedSparse;
  st.oplog_type = petuum::Sparse;
  st.process_cache_capacity = 1;
  st.oplog_capacity = 1;
  st.no_oplog_replay = true;
  if (!petuum::PSTableGroup::CreateTable(kSummaryTable, st)) fail("summary table");

  petuum::ClientTableConfig lt;
  petuum::InitTableConfig(&lt);
  lt.table_info.table_staleness = staleness;
  lt.table_info.oplog_dense_serialized = false;
  lt.table_info.row_capacity = 3;
  lt.table_info.dense_row_oplog_capacity = 3;
  lt.table_info.row_type = kDenseRowDoubleTypeID;
  lt.table_info.server_push_row_upper_bound = 1;
  lt.process_storage_type = petuum::BoundedSparse;
  lt.oplog_type = petuum::Sparse;
  lt.process_cache_capacity = num_iterations;
  lt.oplog_capacity = num_iterations;
  if (!petuum::PSTableGroup::CreateTable(kLLHTable, lt)) fail("llh table");
  petuum::PSTableGroup::CreateTableDone();

  std::vector<std::thread> threads;
  Barrier barrier(num_threads);
  for (int t = 0; t < num_threads; ++t) threads.emplace_back(Worker, t, &barrier);
  for (auto &th : threads) th.join();
  petuum::PSTableGroup::ShutDown();
  return 0;
}
