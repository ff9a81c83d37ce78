// Host batch builder for pre-tokenized item sequences (include/recformer_host.h).
//
// One pass per sequence over the CSR item store: the newest max_items-1 items (the reference
// reverses the past...present list and truncates it, tokenization.py:70-71) are walked
// newest-first, their tokens copied into the output row until max_tokens (:93-95), then the
// row tail is padded (:134-138). Pure integer copies; no per-token allocation.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "../../../include/recformer_host.h"

namespace {

thread_local char g_err[512];

int fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return 1;
}

// items of sequence b, newest first, at most max_items - 1 of them (the <s> slot is the 0th
// item position, models.py item_position_embeddings has max_items rows)
struct SeqView {
  const int64_t* items;
  int64_t n;
};

inline SeqView seq_view(int b, const int64_t* seq_off, const int64_t* seq_items, int max_items) {
  const int64_t n = seq_off[b + 1] - seq_off[b];
  return {seq_items + seq_off[b], std::min<int64_t>(n, std::max(max_items - 1, 0))};
}

int check_common(int B, const int64_t* seq_off, const int64_t* seq_items, int64_t n_items,
                 const int64_t* item_off, int max_items, int max_tokens) {
  if (B < 0 || max_items < 1 || max_tokens < 1) return fail("rf_collate: bad sizes B=%d max_items=%d max_tokens=%d", B, max_items, max_tokens);
  if (B > 0 && (!seq_off || !item_off)) return fail("rf_collate: null pointer");
  for (int b = 0; b < B; ++b) {
    if (seq_off[b + 1] < seq_off[b]) return fail("rf_collate: seq_off not monotone at %d", b);
    for (int64_t k = seq_off[b]; k < seq_off[b + 1]; ++k)
      if (seq_items[k] < 0 || seq_items[k] >= n_items)
        return fail("rf_collate: item index %lld out of range [0, %lld)", (long long)seq_items[k], (long long)n_items);
  }
  return 0;
}

}  // namespace

extern "C" {

const char* rf_host_last_error(void) { return g_err; }

int rf_collate_lengths(int B, const int64_t* seq_off, const int64_t* seq_items, int64_t n_items,
                       const int64_t* item_off, int max_items, int max_tokens, int32_t* out_len) {
  if (int rc = check_common(B, seq_off, seq_items, n_items, item_off, max_items, max_tokens)) return rc;
  if (B > 0 && !out_len) return fail("rf_collate_lengths: null output");
  for (int b = 0; b < B; ++b) {
    const SeqView s = seq_view(b, seq_off, seq_items, max_items);
    int64_t len = 1;  // <s>
    // reversed order: the newest item is seq[n-1]
    for (int64_t k = 0; k < s.n && len < max_tokens; ++k) {
      const int64_t it = s.items[(seq_off[b + 1] - seq_off[b]) - 1 - k];
      len += item_off[it + 1] - item_off[it];
    }
    out_len[b] = (int32_t)std::min<int64_t>(len, max_tokens);
  }
  return 0;
}

int rf_collate_fill(int B, int L, const int64_t* seq_off, const int64_t* seq_items, int64_t n_items,
                    const int64_t* item_off, const int32_t* tok_ids, const int32_t* tok_types,
                    int max_items, int max_tokens, int bos_id, int pad_id, int64_t* input_ids,
                    int64_t* item_position_ids, int64_t* token_type_ids, int64_t* attention_mask,
                    int64_t* global_attention_mask) {
  if (int rc = check_common(B, seq_off, seq_items, n_items, item_off, max_items, max_tokens)) return rc;
  if (L < 1) return fail("rf_collate_fill: L=%d", L);
  if (B > 0 && (!tok_ids || !tok_types || !input_ids || !item_position_ids || !token_type_ids ||
                !attention_mask || !global_attention_mask))
    return fail("rf_collate_fill: null pointer");
  for (int b = 0; b < B; ++b) {
    const int64_t nseq = seq_off[b + 1] - seq_off[b];
    const SeqView s = seq_view(b, seq_off, seq_items, max_items);
    int64_t* ids = input_ids + (int64_t)b * L;
    int64_t* ip = item_position_ids + (int64_t)b * L;
    int64_t* tt = token_type_ids + (int64_t)b * L;
    int64_t* am = attention_mask + (int64_t)b * L;
    int64_t* gm = global_attention_mask + (int64_t)b * L;
    const int64_t cap = std::min<int64_t>(max_tokens, L);
    int64_t t = 0;
    ids[0] = bos_id;  // tokenization.py:74-76
    ip[0] = 0;
    tt[0] = 0;
    t = 1;
    for (int64_t k = 0; k < s.n && t < cap; ++k) {
      const int64_t it = s.items[nseq - 1 - k];
      const int64_t a = item_off[it], e = std::min<int64_t>(item_off[it + 1], a + (cap - t));
      for (int64_t j = a; j < e; ++j, ++t) {
        ids[t] = tok_ids[j];
        tt[t] = tok_types[j];
        ip[t] = k + 1;  // :91 item_idx + 1 (0 is <s>)
      }
    }
    if (t > L) return fail("rf_collate_fill: sequence %d needs %lld > L=%d", b, (long long)t, L);
    for (int64_t j = 0; j < t; ++j) {  // :97-99
      am[j] = 1;
      gm[j] = 0;
    }
    gm[0] = 1;
    for (int64_t j = t; j < L; ++j) {  // :134-138
      ids[j] = pad_id;
      ip[j] = max_items - 1;
      tt[j] = 3;
      am[j] = 0;
      gm[j] = 0;
    }
  }
  return 0;
}

}  // extern "C"
