// Host-side sanitizer test for the native runtime cores (built with
// -fsanitize=address,undefined by tests/unit/test_native_sanitizers.py; GPU sanitizers are not
// available on this pool, so the CPU cores are exercised here).
//
// Covers: BlockManagerCore alloc/free/preempt churn against a shadow model, pack_step layout
// and bounds errors; AES-GCM seal/open round trips, tamper and short-input errors.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>

#include "runtime/block_manager.h"
#include "security/aes_gcm_core.h"

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "%s:%d CHECK(%s)\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

template <class E, class F>
static bool throws(F&& f) {
  try {
    f();
  } catch (const E&) {
    return true;
  }
  return false;
}

static void test_block_manager_churn() {
  const int64_t NB = 257;
  const int BS = 16;
  pk::BlockManagerCore bm(NB, BS, 4);
  std::mt19937_64 rng(1234);
  std::unordered_map<int64_t, int64_t> len;  // shadow: seq -> tokens
  for (int it = 0; it < 20000; ++it) {
    const int op = static_cast<int>(rng() % 4);
    const int64_t seq = static_cast<int64_t>(rng() % 64);
    if (op < 3) {
      const int64_t grow = 1 + static_cast<int64_t>(rng() % 80);
      const int64_t total = (len.count(seq) ? len[seq] : 0) + grow;
      const bool fits = bm.needed(seq, total) <= bm.num_free();
      const bool ok = bm.allocate(seq, total);
      CHECK(ok == fits);
      if (ok) len[seq] = total;
    } else {
      bm.free_seq(seq);
      len.erase(seq);
    }
    if (it % 997 == 0) {
      std::set<int32_t> used;
      int64_t held = 0;
      for (auto& kv : len) {
        auto t = bm.table(kv.first);
        CHECK(static_cast<int64_t>(t.size()) >= bm.blocks_for(kv.second));
        for (int32_t b : t) {
          CHECK(b >= 0 && b < NB);
          CHECK(used.insert(b).second);  // no block owned twice
        }
        held += static_cast<int64_t>(t.size());
      }
      CHECK(held + bm.num_free() == NB);
    }
  }
  for (auto& kv : len) bm.free_seq(kv.first);
  CHECK(bm.num_free() == NB);
  CHECK(bm.num_seqs() == 0);
  CHECK(!bm.can_allocate(999, (NB - 3) * BS, true));  // watermark respected
  CHECK(bm.can_allocate(999, (NB - 4) * BS, true));
}

// Prefix caching under ASan/UBSan: sequences over 4 shared token prefixes are admitted through
// match_prefix / commit_prefix, grown, and freed at random; refcounts must equal table
// membership, free + referenced must equal the pool, and the LRU eviction path is exercised
// because the pool is far smaller than the working set.
static void test_prefix_cache_churn() {
  const int64_t NB = 64;
  const int BS = 8;
  pk::BlockManagerCore bm(NB, BS, 0, true);
  std::mt19937_64 rng(99);
  std::vector<std::vector<uint64_t>> pref(4, std::vector<uint64_t>(4));
  std::vector<std::vector<int32_t>> ptoks(4, std::vector<int32_t>(4 * BS));
  for (int p = 0; p < 4; ++p) {
    for (int i = 0; i < 4 * BS; ++i) ptoks[p][i] = p * 1000 + (i % 7);
    CHECK(bm.prefix_hashes(ptoks[p].data(), 4 * BS, pref[p].data(), 4) == 4);
  }
  std::unordered_map<int64_t, int64_t> len;
  for (int it = 0; it < 20000; ++it) {
    const int op = static_cast<int>(rng() % 3);
    const int64_t seq = static_cast<int64_t>(rng() % 24);
    if (op == 0 && !len.count(seq)) {
      const int p = static_cast<int>(rng() % 4);
      const auto& h = pref[p];
      const int64_t got = bm.match_prefix(seq, h.data(), ptoks[p].data(), 4 * BS, 3);
      if (bm.allocate(seq, 4 * BS)) {
        bm.commit_prefix(seq, h.data(), ptoks[p].data(), 4 * BS, 4);
        len[seq] = 4 * BS;
      } else {
        bm.free_seq(seq);
        CHECK(got >= 0);
      }
    } else if (op == 1 && len.count(seq)) {
      const int64_t total = len[seq] + 1 + static_cast<int64_t>(rng() % 40);
      if (bm.allocate(seq, total)) len[seq] = total;
    } else if (op == 2) {
      bm.free_seq(seq);
      len.erase(seq);
    }
    if (it % 499 == 0) {
      std::unordered_map<int32_t, int> refs;
      for (auto& kv : len)
        for (int32_t b : bm.table(kv.first)) ++refs[b];
      for (auto& kv : refs) CHECK(bm.ref_count(kv.first) == kv.second);
      CHECK(static_cast<int64_t>(refs.size()) + bm.num_free() == NB);
    }
  }
  for (auto& kv : len) bm.free_seq(kv.first);
  CHECK(bm.num_free() == NB);
  CHECK(bm.prefix_hits() > 0);
  bm.reset_prefix_cache();
  CHECK(bm.num_cached() == 0 && bm.num_free() == NB);
}

static void test_pack() {
  pk::BlockManagerCore bm(32, 4, 0);
  CHECK(bm.allocate(7, 6));   // 2 blocks
  CHECK(bm.allocate(9, 1));   // 1 block
  const int64_t sid[2] = {7, 9};
  const int32_t nc[2] = {2, 0}, nn[2] = {4, 1};
  const int32_t tok[5] = {10, 11, 12, 13, 20};
  int32_t ids[5], pos[5], slot[5], bt[2 * 3], cl[2], cu[3];
  const int64_t T = bm.pack(2, sid, nc, nn, tok, ids, pos, slot, bt, 2, 3, 3, cl, cu);
  CHECK(T == 5);
  auto t7 = bm.table(7), t9 = bm.table(9);
  for (int j = 0; j < 4; ++j) {
    const int p = 2 + j;
    CHECK(pos[j] == p);
    CHECK(ids[j] == tok[j]);
    CHECK(slot[j] == t7[p / 4] * 4 + p % 4);
  }
  CHECK(slot[4] == t9[0] * 4);
  CHECK(bt[0] == t7[0] && bt[1] == t7[1] && bt[2] == 0);
  CHECK(bt[3] == t9[0] && bt[4] == 0 && bt[5] == 0);
  CHECK(cl[0] == 6 && cl[1] == 1);
  CHECK(cu[0] == 0 && cu[1] == 4 && cu[2] == 5);
  const int64_t missing[1] = {42};
  CHECK(throws<std::runtime_error>([&] { bm.pack(1, missing, nc, nn, tok, ids, pos, slot, bt, 2, 3, 3, cl, cu); }));
  const int32_t nn_big[1] = {9};
  CHECK(throws<std::runtime_error>([&] { bm.pack(1, sid, nc, nn_big, tok, ids, pos, slot, bt, 2, 3, 3, cl, cu); }));
  CHECK(throws<std::invalid_argument>([&] { bm.pack(2, sid, nc, nn, tok, ids, pos, slot, bt, 1, 3, 3, cl, cu); }));
  CHECK(throws<std::invalid_argument>([] { pk::BlockManagerCore bad(0, 4, 0); }));
}

static void test_aes() {
  using namespace pk_aes;
  std::string key(kKeyLen, '\0');
  for (int i = 0; i < kKeyLen; ++i) key[i] = static_cast<char>(i * 7 + 1);
  auto ctx = new_ctx();
  std::mt19937 rng(7);
  for (int n : {0, 1, 15, 16, 17, 255, 4096}) {
    std::string pt(n, '\0');
    for (auto& c : pt) c = static_cast<char>(rng());
    const std::string ct = seal(ctx.get(), key, pt);
    CHECK(ct.size() == pt.size() + kNonceLen + kTagLen);
    CHECK(open(ctx.get(), key, ct) == pt);
    std::string bad = ct;
    bad[bad.size() / 2] ^= 1;
    CHECK(throws<std::invalid_argument>([&] { open(ctx.get(), key, bad); }));
  }
  const std::string a = seal(ctx.get(), key, "same"), b = seal(ctx.get(), key, "same");
  CHECK(a != b);  // fresh nonce per message
  CHECK(throws<std::invalid_argument>([&] { open(ctx.get(), key, "short"); }));
  CHECK(throws<std::invalid_argument>([&] { open(ctx.get(), key, std::string(kNonceLen + 3, 'x')); }));
  CHECK(throws<std::invalid_argument>([] { validate_key("short-key"); }));
  std::string other = key;
  other[0] ^= 0x55;
  CHECK(throws<std::invalid_argument>([&] { open(ctx.get(), other, a); }));
}

int main() {
  test_block_manager_churn();
  test_prefix_cache_churn();
  test_pack();
  test_aes();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("native tests OK\n");
  return 0;
}
