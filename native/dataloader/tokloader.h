// Native token-shard data loader for the training workload (C ABI, loaded with ctypes).
//
// Shards are flat binary files of token ids (uint16 or uint32), optionally with the 1 KiB llm.c
// header (int32 magic 20240520, version 1 = uint16 / 2 = uint32, token count).  Every shard is
// memory-mapped; the corpus is cut into non-overlapping windows of seq_len + 1 tokens (input and
// shifted target), and each epoch visits all windows in a seeded random order.  Rank r of W takes
// windows [(i * W + r) * batch, ... + batch) of the epoch order for its batch i, so ranks never
// share a window and a job resumes exactly from a batch index (tl_seek).  A background thread keeps
// `prefetch` batches assembled ahead of the consumer.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct TokLoader TokLoader;

// NULL on error (message in err).  token_bytes: 0 = from the llm.c header, else 2 or 4 for
// headerless shards.
TokLoader* tl_open(const char* const* paths, int n_paths, int token_bytes, int seq_len, int batch, uint64_t seed,
                   int rank, int world, int prefetch, char* err, int err_len);
// Copy the next batch (batch x (seq_len + 1) int32 tokens, row-major) and its index; 0 on success.
int tl_next(TokLoader* l, int32_t* out, uint64_t* batch_index);
// Position the loader so that the next tl_next returns batch `batch_index` (resume).
void tl_seek(TokLoader* l, uint64_t batch_index);
uint64_t tl_num_windows(const TokLoader* l);
uint64_t tl_num_tokens(const TokLoader* l);
uint64_t tl_batches_per_epoch(const TokLoader* l);
void tl_close(TokLoader* l);

#ifdef __cplusplus
}
#endif
