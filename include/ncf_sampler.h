/*
 * ncf_sampler.h -- C ABI of libncf_sampler.so, the host-side negative sampler.
 *
 * Replaces the pure-Python NCFData.ng_sample (reference src/data/datasets.py:53-69)
 * with a C++ loop that consumes NumPy's *global legacy* MT19937 stream word for
 * word: state in/out uses numpy.random.get_state()'s layout (key[624], pos),
 * randint(n) is masked rejection over 32-bit outputs, and membership is the
 * training set of (user, item) pairs (the dok_matrix of datasets.py:23-24).
 * Output is bit-identical to the reference for identical seeds.
 */
#ifndef NCF_SAMPLER_H
#define NCF_SAMPLER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Build the membership index over the training positives (file order). */
void *ncf_sampler_create(const int32_t *users, const int32_t *items, int64_t n_pos, int32_t n_users,
                         int32_t n_items);
void ncf_sampler_destroy(void *s);

/* 1 if (u, i) is a training positive ((u, j) in train_mat, datasets.py:61). */
int ncf_sampler_contains(const void *s, int32_t u, int32_t i);

/* np.random.seed(seed) for the legacy generator: key[624], *pos = 624. */
void ncf_mt_seed(uint32_t seed, uint32_t *key, int32_t *pos);

/*
 * Continue the MT19937 stream (key, pos) by n tempered 32-bit words into out
 * (NULL: advance only) -- the words numpy's legacy RandomState and torch's CPU
 * generator (torch.Generator.manual_seed(s): key = ncf_mt_seed(s & 0xffffffff))
 * draw next.  The device epoch pipeline (ncf_sample_negatives, ncf_randperm in
 * ncf_hip.h) consumes them.
 */
void ncf_mt_words(uint32_t *key, int32_t *pos, int64_t n, uint32_t *out);

/*
 * One ng_sample() pass: for every positive p (file order) and t < num_ng, draw
 * j = randint(num_item) until (user[p], j) is not a positive; out_items[p*num_ng+t] = j.
 * key/pos: the MT19937 state, advanced in place.  Returns the number of 32-bit
 * words consumed, or -1 on bad arguments.
 */
int64_t ncf_sampler_sample(const void *s, int32_t num_item, int32_t num_ng, uint32_t *key, int32_t *pos,
                           int32_t *out_items);

#ifdef __cplusplus
}
#endif
#endif /* NCF_SAMPLER_H */
