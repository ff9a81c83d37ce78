/*
 * librecformer_host — C ABI of the host-side batch builder.
 *
 * Replaces the per-token Python loops of the reference's input pipeline for pre-tokenized
 * items: RecformerTokenizer.encode(items, encode_item=False) (recformer/tokenization.py:64-105)
 * + RecformerTokenizer.padding (tokenization.py:108-152), as driven by
 * FinetuneDataCollatorWithPadding / EvalDataCollatorWithPadding (collator.py:245-385:
 * extract_features -> encode_features -> padding -> torch.LongTensor).
 *
 * Item store: the reference's `tokenized_items` dict {item: [input_ids, token_type_ids]}
 * (finetune.py:239-245) flattened to CSR form: item i's tokens are tok_ids[item_off[i] ..
 * item_off[i+1]) with types tok_types[...] (input_ids and token_type_ids of equal length).
 * A batch is B sequences of item indices in the reference's order (past ... present),
 * sequence b = seq_items[seq_off[b] .. seq_off[b+1]).
 *
 * Outputs are the five (B, L) int64 row-major arrays the collators hand to the model
 * (input_ids, item_position_ids, token_type_ids, attention_mask, global_attention_mask),
 * written straight into caller-owned (e.g. pinned) host memory. Plain host pointers; no
 * allocation; re-entrant (distinct batches may be built on different threads). Return 0 on
 * success, else rf_host_last_error() holds a thread-local message.
 */
#ifndef RECFORMER_HOST_H
#define RECFORMER_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* rf_host_last_error(void);

/* Encoded length of every sequence (tokenization.py:70-95: reverse, keep the newest
 * max_items-1 items, <s> + their tokens, truncate to max_tokens). out_len: B int32. */
int rf_collate_lengths(int B, const int64_t* seq_off, const int64_t* seq_items, int64_t n_items,
                       const int64_t* item_off, int max_items, int max_tokens, int32_t* out_len);

/* Fill the (B, L) arrays: encode (tokenization.py:64-105) then pad to L (tokenization.py:
 * 134-138: ids <- pad_id, item position <- max_items - 1, type <- 3, masks <- 0). L must be
 * >= every encoded length (rf_collate_lengths; the reference pads to their max, or to
 * max_tokens with pad_to_max). */
int rf_collate_fill(int B, int L, const int64_t* seq_off, const int64_t* seq_items, int64_t n_items,
                    const int64_t* item_off, const int32_t* tok_ids, const int32_t* tok_types,
                    int max_items, int max_tokens, int bos_id, int pad_id, int64_t* input_ids,
                    int64_t* item_position_ids, int64_t* token_type_ids, int64_t* attention_mask,
                    int64_t* global_attention_mask);

#ifdef __cplusplus
}
#endif
#endif
