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

/*
 * The general form: the draw loop runs over pos_users (features_ps in file order,
 * datasets.py:57) while membership is the (mem_users, mem_items) pairs -- the keys of
 * train_mat (datasets.py:61), which may hold pairs beyond the positives.
 */
void *ncf_sampler_create2(const int32_t *pos_users, int64_t n_pos, const int32_t *mem_users,
                          const int32_t *mem_items, int64_t n_mem, int32_t n_users, int32_t n_items);

/*
 * Host threads of the sampler's pass (default: NCF_SAMPLER_THREADS, else
 * min(16, 3/4 of the CPUs)).  1 runs the sequential pass; > 1 the parallel pass
 * (bitset membership): the word stream in chunks from MT19937 jump-ahead states,
 * the walk as a sequential chain over per-run membership windows tabulated in
 * parallel.  Both give the same negatives and end state.  0, or -1 on bad args.
 */
int ncf_sampler_set_threads(void *s, int32_t threads);

/*
 * Counters of the sampler: out[0..n) = parallel passes, sequential passes, runs
 * the chain walked directly (outside their window), parallel passes redone
 * sequentially, threads, blocks of runs, and of the last parallel pass the ns of
 * words / walk / end state / chain and the tabulated window bits.
 */
int ncf_sampler_stats(const void *s, int64_t *out, int32_t n);
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
 * j = randint(num_item) until (user[p], j) is not a member; out_items[p*num_ng+t] = j.
 * key/pos: the MT19937 state, advanced in place.  Returns the number of 32-bit
 * words consumed, -1 on bad arguments, -2 if some user owns every item in
 * [0, num_item) (the reference's redraw loop would never end).
 */
int64_t ncf_sampler_sample(const void *s, int32_t num_item, int32_t num_ng, uint32_t *key, int32_t *pos,
                           int32_t *out_items);

/*
 * MT19937 jump-ahead: key[624] (a generator's array, i.e. the 624-word window of
 * its untempered stream) becomes the window J words later: x^J mod the
 * generator's minimal polynomial (Berlekamp-Massey, once per process) applied
 * as a correlation with the next ~20K words.  For J a multiple of 624 this is
 * exactly the array numpy / torch hold after J more draws.  0, or -1.
 */
int ncf_mt_jump(uint32_t *key, int64_t J);

/*
 * Parallel ncf_mt_words (torch's randperm words, numpy's stream): a pool of
 * `threads` host threads; each fills a 624-aligned chunk of the n words from the
 * state jumped to it.  Same words and end state as ncf_mt_words.
 */
void *ncf_words_create(int32_t threads);
void ncf_words_destroy(void *h);
int ncf_words_fill(void *h, uint32_t *key, int32_t *pos, int64_t n, uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif /* NCF_SAMPLER_H */
