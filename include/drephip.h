/*
 * drephip.h -- C ABI of libdrephip.so, the MI355X (gfx950) implementation of
 * dRep's primary-clustering hot path: Mash sketch + all-vs-all Mash dist.
 *
 * The reference does this step by shelling out to the external Mash binary
 * (drep/d_cluster.py:481-596, all_vs_all_MASH).  Each entry point below names
 * the reference interface it replaces.  Conventions:
 *   - every function returns 0 on success and a negative DREPHIP_ERR_* code on
 *     failure (the reference ignored mash's exit codes, drep/__init__.py:44-48;
 *     here failures are reported) -- drephip_last_error() gives the message
 *     (thread-local);
 *   - host buffers are owned by the caller (numpy arrays via ctypes); device
 *     memory passed in (d_ prefix) is owned by the caller too; the library owns
 *     its own device scratch, kept in the context;
 *   - calls are blocking and a context is single-caller; no C++ exception
 *     crosses the ABI.
 *
 * Sketch definition (bit-exact with `mash sketch -k 21 -s S`, seed 42):
 *   canonical k-mer (memcmp(fwd, revcomp) <= 0 ? fwd : revcomp) hashed with
 *   MurmurHash3_x64_128(seed).h1 over its ASCII bytes; k-mers containing a
 *   non-ACGT byte (after upper-casing) or spanning two records are skipped;
 *   sketch = the s smallest distinct hashes, ascending, one sketch per file.
 * hashes_out rows are s wide; entries past nhash are UINT64_MAX.
 *
 * Pair output: condensed upper triangle (i < j, row-major; scipy squareform
 * order): index(i, j) = i*N - i*(i+1)/2 + (j - i - 1).
 *   common = Mash's shared-hash count (the "c" of "c/denom" in MASH_table.tsv),
 *   denom  = s when both sketches are full, else min(s, |A u B|).
 */
#ifndef DREPHIP_H
#define DREPHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DREPHIP_OK               0
#define DREPHIP_ERR_ARG         -1
#define DREPHIP_ERR_HIP         -2
#define DREPHIP_ERR_IO          -3
#define DREPHIP_ERR_NOMEM       -4
#define DREPHIP_ERR_UNSUPPORTED -5
#define DREPHIP_ERR_INTERNAL    -6

typedef struct drephip_ctx drephip_ctx;

/* Library/ABI version (major*10000 + minor*100 + patch). */
int drephip_version(void);

/* Build identity: "src=<sha256 of the library's sources>;arch=gfx950;extra=<A/B
 * build flags>" -- the digest is computed by drep_amd/csrc/Makefile over
 * include/drephip.h and drep_amd/csrc/ (drep_amd/_lib.py:source_digest restates
 * it), so a caller can prove which sources the loaded library was built from. */
const char *drephip_build_id(void);

/* Last error message of the calling thread ("" if none). */
const char *drephip_last_error(void);

/* Number of visible HIP devices. */
int drephip_device_count(int *n);

/* Create a context on HIP device `device` for k-mer size k (1..32), sketch
 * size s (1..DREPHIP_MAX_SKETCH) and Murmur seed.
 * Replaces: the `mash` executable lookup + parameters,
 *   drep/d_cluster.py:499-515 (MASH_sketch, exe_loc/get_exe), drep/__init__.py:88-101. */
int drephip_create(int device, int k, uint32_t s, uint32_t seed, drephip_ctx **out);
int drephip_destroy(drephip_ctx *ctx);

/* Largest supported sketch size. */
uint32_t drephip_max_sketch(void);

/* ---------------------------------------------------------------- layout
 * Packed genome set in HBM: 2-bit base codes (A0 C1 G2 T3), 16 bases per
 * uint32 (base p at bits 2*(p%16)); validity bitmap, 32 bases per uint32 (bit
 * p%32 of word p/32).  Genome g occupies bases [base_off[g], base_off[g] +
 * padded[g]); base_off[0] = tile, base_off and padded are multiples of
 * drephip_tile_bases(); records are separated by one invalid base and every
 * genome is followed by at least one invalid base; bases [0, tile) are
 * invalid. */
uint64_t drephip_tile_bases(void);

/* Padded size (in bases) of a genome whose records have the given lengths. */
uint64_t drephip_padded_bases(const uint64_t *rec_len, uint32_t n_rec);

/* Parse a FASTA file (plain or gzip; kseq semantics as in Mash) -- what
 * `mash sketch <fasta>` reads (drep/d_cluster.py:543-544).  Outputs the sum of
 * record lengths, the padded size, the record count and the number of valid
 * k-mer positions. */
int drephip_fasta_info(const char *path, int k, uint64_t *length, uint64_t *padded,
                       uint32_t *n_records, uint64_t *n_kmers);

/* Pack a FASTA into the layout at base offset `base_off` of caller-owned host
 * arrays (codes/valid sized for at least base_off+padded bases; the genome's
 * padded region must be zero on entry). */
int drephip_fasta_pack(const char *path, int k, uint32_t *codes, uint32_t *valid,
                       uint64_t base_off, uint64_t cap_bases, uint64_t *length,
                       uint64_t *n_kmers);

/* ---------------------------------------------------------------- sketch
 * Replaces: `mash sketch <fa> -s S -o <out>` per genome on a thread pool
 * (drep/d_cluster.py:531-549, drep/__init__.py:53-59) and `mash paste`
 * (d_cluster.py:551-567): one call sketches a whole genome set into one
 * row-major uint64[n_genomes][s] matrix.
 * Input: concatenated sequence bytes (any case) of every record of every
 * genome; rec_off[n_rec+1] record boundaries into seq; genome g owns records
 * [genome_rec_off[g], genome_rec_off[g+1]). */
int drephip_sketch(drephip_ctx *ctx, const uint8_t *seq, const uint64_t *rec_off, uint32_t n_rec,
                   const uint64_t *genome_rec_off, uint32_t n_genomes,
                   uint64_t *hashes_out, uint32_t *nhash_out, uint64_t *length_out);

/* Same, reading FASTA files (kseq semantics, plain or gzip) on `threads` CPU
 * threads (0 = all).  Files are read and packed in batches of ~1 Gbase into
 * two pinned host buffers by a producer thread while the calling thread copies
 * the previous batch to the device and sketches it (host ingest and GPU work
 * overlap).  drephip_last_ingest_stats reports the split. */
int drephip_sketch_files(drephip_ctx *ctx, const char *const *paths, uint32_t n_genomes,
                         int threads, uint64_t *hashes_out, uint32_t *nhash_out,
                         uint64_t *length_out);

/* Timing of the last drephip_sketch_files call on this context (seconds):
 * host read + pack summed over batches, device copy + sketch summed over
 * batches, the whole call's wall time, and the number of batches.  With the
 * overlap, wall ~ produce + the last batch's device work. */
int drephip_last_ingest_stats(drephip_ctx *ctx, double *produce_s, double *gpu_s, double *wall_s,
                              uint32_t *batches);

/* Host phases of the last drephip_sketch_files call, summed over the worker
 * threads (seconds): FASTA read + parse (gzip inflate included) and the 2-bit
 * pack; and the number of genomes whose span outgrew the region their file
 * size (or gzip ISIZE) reserved, repacked at the end of their batch. */
int drephip_last_ingest_phases(drephip_ctx *ctx, double *read_thread_s, double *pack_thread_s,
                               uint32_t *overflow);

/* Device-resident sketch: packed genome set already in HBM (see layout).
 * h_base_off/h_padded/h_nkmers are host arrays of n_genomes entries
 * (h_nkmers: valid k-mer positions, used only to seed the candidate
 * threshold).  d_hashes: uint64[n_genomes][s]; d_nhash: uint32[n_genomes].
 * stream: a hipStream_t; 0 is the HIP null stream (as everywhere in HIP).
 * Every device-pointer entry point runs on the stream it is given, so it is
 * ordered after work the caller queued there.  Blocking. */
int drephip_sketch_device(drephip_ctx *ctx, const uint32_t *d_codes, const uint32_t *d_valid,
                          const uint64_t *h_base_off, const uint64_t *h_padded,
                          const uint64_t *h_nkmers, uint32_t n_genomes,
                          uint64_t *d_hashes, uint32_t *d_nhash, void *stream);

/* Same as drephip_sketch_device, but returns once the first threshold round
 * is queued, without waiting for it: work the caller queues next on `stream`
 * (the sketch all-gather, drephip_allpairs_device) runs right behind it.
 * d_hashes/d_nhash are final only after drephip_sketch_wait, which must be
 * called before the next sketch call on this context: until then every other
 * sketch call fails with DREPHIP_ERR_ARG (the pending check is kept).  The
 * inputs (d_codes, d_valid) must stay unchanged until the wait, which may
 * rerun the call from them. */
int drephip_sketch_device_async(drephip_ctx *ctx, const uint32_t *d_codes, const uint32_t *d_valid,
                                const uint64_t *h_base_off, const uint64_t *h_padded,
                                const uint64_t *h_nkmers, uint32_t n_genomes,
                                uint64_t *d_hashes, uint32_t *d_nhash, void *stream);

/* Completes a drephip_sketch_device_async call: waits for its stream, checks
 * every genome's first-round status and, if any genome needs another
 * threshold round (a genome with fewer distinct k-mers than expected, or
 * heavy repeats), reruns the whole call synchronously and sets *redone = 1:
 * anything the caller computed from the sketches in between must then be
 * recomputed.  *redone = 0 otherwise (also when nothing is pending).  The
 * sketch kernels' drephip_last_kernel_ms entries (0, 1) are set here. */
int drephip_sketch_wait(drephip_ctx *ctx, int *redone);

/* Bench/test input: write synthetic genomes g0..g0+n-1 (each length L, one
 * record; family = g / family_size) into the packed layout with
 * genome i at base_off = tile + i*drephip_padded_bases(&L, 1).
 * d_codes/d_valid must hold tile + n*padded bases. */
int drephip_synth_device(drephip_ctx *ctx, uint64_t seed, uint32_t g0, uint32_t n,
                         uint32_t family_size, uint64_t L, uint32_t *d_codes, uint32_t *d_valid,
                         void *stream);

/* ---------------------------------------------------------------- dist
 * Replaces: `mash dist -p P ALL.msh ALL.msh > MASH_table.tsv`
 * (drep/d_cluster.py:569-573) for the integer part of every row: the shared-
 * hash count and its denominator.  Distances are a pure function of
 * (common, denom) and are formed on the host (drephip_distance_lut).
 * Input: N rows of s hashes, ascending and distinct; entries past nhash[i] are
 * UINT64_MAX (as drephip_sketch* write them -- the kernels read whole rows;
 * drephip_allpairs checks this, the device entry points assume it). */
int drephip_allpairs(drephip_ctx *ctx, const uint64_t *hashes, const uint32_t *nhash, uint32_t N,
                     uint16_t *common_out, uint16_t *denom_out /* nullable */);

/* drephip_allpairs restricted to rows [row0, row1) of the upper triangle
 * (columns row+1..N-1): common_out/denom_out receive the condensed segment
 * that starts at index(row0, row0+1), i.e. row0*N - row0*(row0+1)/2.  One call
 * per device (one context each) splits the triangle across GPUs inside one
 * process -- the multi-device form of the same `mash dist` step. */
int drephip_allpairs_rows(drephip_ctx *ctx, const uint64_t *hashes, const uint32_t *nhash, uint32_t N,
                          uint32_t row0, uint32_t row1, uint16_t *common_out, uint16_t *denom_out /* nullable */);

/* Device-resident all-pairs over rows [row0, row1) of the upper triangle
 * (columns row+1..N-1).  d_common/d_denom receive the condensed segment that
 * starts at index(row0, row0+1).  d_denom may be NULL. Blocking. */
int drephip_allpairs_device(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash,
                            uint32_t N, uint32_t row0, uint32_t row1, uint16_t *d_common,
                            uint16_t *d_denom, void *stream);

/* Same as drephip_allpairs_device, but on the whole-row table path (s <=
 * 2048) it returns once the kernels are queued: the host can queue the next
 * step's work while they run.  The output is final once the work queued on
 * `stream` before and by this call has run (the kernels handle every row
 * themselves, including a row whose table cannot be built, which they merge
 * literally); drephip_allpairs_wait (or any later all-pairs or linkage call on
 * this context) waits for it.  Other paths run synchronously (the wait is
 * then a no-op).  Kernel timings of a deferred call are not recorded. */
int drephip_allpairs_device_async(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash,
                                  uint32_t N, uint32_t row0, uint32_t row1, uint16_t *d_common,
                                  uint16_t *d_denom, void *stream);
int drephip_allpairs_wait(drephip_ctx *ctx);

/* Reference all-pairs kernel (one lane per pair, literal Mash merge loop).
 * Same contract as drephip_allpairs_device; slower; used for cross-checks. */
int drephip_allpairs_merge_device(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash,
                                  uint32_t N, uint32_t row0, uint32_t row1, uint16_t *d_common,
                                  uint16_t *d_denom, void *stream);

/* Mash distance for common = 0..denom at the given denominator (host, libm):
 * J = c/denom; d = c==denom ? 0 : c==0 ? 1 : min(1, -ln(2J/(1+J))/k).
 * Reference: the "dist" column of MASH_table.tsv parsed at d_cluster.py:581. */
int drephip_distance_lut(int k, uint32_t denom, double *lut /* denom+1 */);

/* MASH_table.tsv as `mash dist -p P ALL.msh ALL.msh > MASH_table.tsv` prints
 * it (drep/d_cluster.py:569-573): for every query q (outer loop) and reference
 * r, "names[r]\tnames[q]\t%g dist\t%g p-value\tcommon/denom\n".  Pairs come
 * from the condensed result (index(i, j), i < j; denom NULL = s for every
 * pair) with their distances and p-values (caller-computed: Mash's formula,
 * drephip_distance_lut; p-values with the binomial tail); a genome against
 * itself prints distance 0, self_pval[q] and self_count[q]/self_count[q].
 * Host only; rows are formatted on `threads` threads (0 = all) and written in
 * order. */
int drephip_write_mash_table(const char *path, const char *const *names, uint32_t N,
                             const uint16_t *common, const uint16_t *denom /* nullable */, uint32_t s,
                             const double *dist, const double *pval, const uint16_t *self_count,
                             const double *self_pval, int threads);

/* All-pairs kernel selection (no CPU path exists; every choice is a HIP kernel
 * with the same bit-exact result):
 *   DREPHIP_AP_AUTO  whole-row LDS tables for s <= 2048, value bands above;
 *   DREPHIP_AP_TABLE k_allpairs_q (s <= 2048);
 *   DREPHIP_AP_BAND  k_allpairs_band, band_cap (1..1024) elements per row per
 *                    band, clamped to the kernel's LDS budget (768; the
 *                    default is the production setting; small caps exercise
 *                    many bands on small sketches in tests);
 *   DREPHIP_AP_MERGE k_allpairs_merge (literal merge, cross-check only). */
#define DREPHIP_AP_AUTO 0
#define DREPHIP_AP_TABLE 1
#define DREPHIP_AP_BAND 2
#define DREPHIP_AP_MERGE 3
int drephip_set_allpairs_path(drephip_ctx *ctx, int path, uint32_t band_cap);

/* The shared-hash screen in front of the table / band kernels (an exact
 * shortcut inside `mash dist`, drep/d_cluster.py:569-573): Mash's merge of two
 * sketches that share no hash is common 0, denominator min(s, |A| + |B|), so
 * the sketch entries are grouped by value (radix sort on the device), the
 * (row tile, column) cells whose genomes share a hash are listed, the kernels
 * run on those only and every other pair is written as no-shared-hash.
 *   DREPHIP_SCREEN_AUTO  on when N >= 4096 and the pair checks the grouping
 *                        implies stay below (pairs x s) / 16 (else the dense
 *                        item plan runs);
 *   DREPHIP_SCREEN_ON    always (unless N x s >= 2^32);
 *   DREPHIP_SCREEN_OFF   never.
 * The environment variable DREPHIP_AP_SCREEN (0/1/2) overrides the mode. */
#define DREPHIP_SCREEN_AUTO 0
#define DREPHIP_SCREEN_ON 1
#define DREPHIP_SCREEN_OFF 2
int drephip_set_allpairs_screen(drephip_ctx *ctx, int mode);
/* The last all-pairs call's screen: whether it replaced the dense plan, the
 * sketch entries grouped, the runs of equal keys, the pair checks, the
 * marked (row tile, column) cells left to the kernels and the pairs sharing
 * exactly one hash that the screen wrote itself.  After
 * drephip_allpairs_device_marked: entries, runs and checks of the hash part
 * this context grouped last. */
int drephip_last_screen_stats(drephip_ctx *ctx, int *used, uint64_t *entries, uint64_t *runs, uint64_t *checks,
                              uint64_t *marked, uint64_t *simple);

/* The sharded screen (a W-way sharded `mash dist`, one rank per GPU): instead
 * of every rank grouping all N x s entries, rank p groups hash part p of W
 * (the p-th of W hash value ranges, cut at the medians over the genomes of
 * each sketch's p/W quantiles, so every rank computes the same cuts: equal
 * hashes lie in one part, and each sketch row -- ascending, as every all-pairs
 * call requires -- holds a part's hashes in one range), marks the (row tile, column) cells of EVERY
 * row from its runs of >= 3 and lists its runs of two; the ranks route the
 * marks to the ranks owning their rows (an all-to-all: RCCL or gloo, the
 * caller's), and each rank screens its own rows from what it received.  Same
 * result as drephip_allpairs_device with the screen on (no light cells).
 * Replaces the per-rank grouping inside the sharded form of
 * drep/d_cluster.py:569-573.
 *
 * drephip_screen_geometry: rows per row tile R (the all-pairs kernels' for
 * this s).  Row tiles count from row 0: tile T holds rows [T R, (T + 1) R).
 * drephip_screen_part: part `part` of `nparts`; *checks = the part's pair
 * checks (their sum over the parts decides the screen: drephip_screen_worth
 * sets *applies when this context screens N genomes at all -- mode, N, N x s --
 * and *use when it would screen them with those checks, as
 * drephip_allpairs_device decides), *n_cells = its marked cell words,
 * *n_records = its runs-of-two records.  Blocking.  Results stay in the
 * context until drephip_screen_part_copy copies them out, each as 4 uint32:
 *   cell   {T, w, bits, 0}: columns 32 w + b (bit b set) of row tile T marked
 *   record {a, b, (i << 16) | j, 0}: genomes a < b hold one hash at positions
 *          i, j (a run of two);
 * route a cell to the rank owning rows T R.., a record to the rank owning row a.
 * drephip_allpairs_device_marked: drephip_allpairs_device over rows
 * [row0, row1) screened from the cells and records given (every part's for
 * these rows; others are ignored).  Rank boundaries on multiples of R keep the
 * marks exact; otherwise a tile straddling a boundary gives both ranks its
 * cells (more kernel work, the same result). */
int drephip_screen_geometry(drephip_ctx *ctx, uint32_t *rows_per_tile);
int drephip_screen_part(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                        uint32_t part, uint32_t nparts, uint64_t *checks, uint32_t *n_cells, uint32_t *n_records,
                        void *stream);
int drephip_screen_part_copy(drephip_ctx *ctx, uint32_t *d_cells, uint32_t *d_records, void *stream);
int drephip_screen_worth(drephip_ctx *ctx, uint32_t N, uint64_t checks, int *applies /* nullable */, int *use);
int drephip_allpairs_device_marked(drephip_ctx *ctx, const uint64_t *d_hashes, const uint32_t *d_nhash, uint32_t N,
                                   uint32_t row0, uint32_t row1, uint16_t *d_common, uint16_t *d_denom,
                                   const uint32_t *d_cells, uint64_t n_cells, const uint32_t *d_records,
                                   uint64_t n_records, void *stream);

/* ---------------------------------------------------------- primary clustering
 * Replaces: scipy.cluster.hierarchy.linkage(squareform(dist), method) in
 * cluster_hierarchical (drep/d_cluster.py:447-453), called from
 * cluster_mash_database (598-630) -- the O(n^2) step of primary clustering.
 * Result: the (n-1) x 4 linkage matrix Z, bit-identical to scipy's (its
 * nn_chain for complete/average/weighted, mst_single_linkage for single,
 * then its stable sort and relabel).  Method codes are scipy's. */
#define DREPHIP_LINK_SINGLE 0
#define DREPHIP_LINK_COMPLETE 1
#define DREPHIP_LINK_AVERAGE 2
#define DREPHIP_LINK_WEIGHTED 6
/* Two paths, chosen per call (drephip_set_linkage_path):
 *  - sparse: when no distance exceeds 1.0 -- Mash's distance of two genomes
 *    sharing no hash is exactly 1.0, the top of its range -- scipy's algorithm
 *    is replayed on the host over the pairs below 1.0 only (one small dense
 *    matrix per connected component of those pairs; the counts path extracts
 *    them on the GPU).  Bit-identical to scipy.  Used automatically when the
 *    per-component matrices fit 2^28 f64 cells (DREPHIP_LINK_SPARSE_CELLS);
 *    when the path is forced (and in drephip_linkage_sparse) components too
 *    large for matrices run scipy's chain over sparse rows instead (no
 *    matrix; host time grows with the rows' lengths: ~1 s at 2x10^4 genomes
 *    with ~100 chance links each);
 *  - dense: the n x n f64 matrix in HBM, one GPU launch per chain step. */
#define DREPHIP_LINK_PATH_AUTO 0
#define DREPHIP_LINK_PATH_DENSE 1
#define DREPHIP_LINK_PATH_SPARSE 2   /* fails (DREPHIP_ERR_UNSUPPORTED) where no sparse form exists */
/* (a new context starts at DREPHIP_LINK_PATH_AUTO, or at the path named by the
 * environment variable DREPHIP_LINK_PATH = auto | dense | sparse) */
int drephip_set_linkage_path(drephip_ctx *ctx, int path);
/* From a host condensed distance vector y (n(n-1)/2 doubles, scipy order). */
int drephip_linkage(drephip_ctx *ctx, const double *y, uint32_t n, int method, double *Z /* (n-1)*4 */);
/* From the device-resident all-pairs output of drephip_allpairs_device (rows
 * 0..n-1 in one segment): distance of pair (i, j) = lut[lut_off[denom] +
 * common] (denom = s when d_denom is NULL; lut_off has s+1 entries, -1 for a
 * denominator that does not occur), placed at row/column perm[i], perm[j] of
 * the linkage input.  The counts are read after all work queued on `stream`
 * (and after a pending drephip_allpairs_device_async on this context).  A pair
 * whose denominator has no table, or whose count exceeds it, fails the call
 * (DREPHIP_ERR_ARG).  Blocking. */
int drephip_linkage_counts_device(drephip_ctx *ctx, const uint16_t *d_common, const uint16_t *d_denom,
                                  uint32_t n, const uint32_t *perm, const double *lut, uint32_t lut_len,
                                  const int32_t *lut_off, int method, double *Z /* (n-1)*4 */, void *stream);

/* From the host n x n float32 matrix the reference's pivot produces
 * (cluster_mash_database, drep/d_cluster.py:619-621: db.pivot(genome1,
 * genome2, dist) -> cluster_hierarchical's squareform -> linkage, 445-453):
 * Z = scipy.cluster.hierarchy.linkage(squareform(M), method).  The matrix is
 * copied to the device, where squareform's checks run (M == M^T element by
 * element, a zero diagonal) and linkage's (finite values), and the f64 linkage
 * input is built from the upper triangle, as squareform takes it.  A failed
 * check fails the call with DREPHIP_ERR_ARG and scipy's message ("Distance
 * matrix 'X' must be symmetric.", "Distance matrix 'X' diagonal must be
 * zero.", "The condensed distance matrix must contain only finite values.").  Dense path;
 * blocking. */
int drephip_linkage_square(drephip_ctx *ctx, const float *M, uint32_t n, int method, double *Z /* (n-1)*4 */);

/* ------------------------------------------------------------ Mdb on the host
 * The N^2-row Mdb table all_vs_all_MASH returns (drep/d_cluster.py:575-596),
 * filled from the condensed all-pairs result without the reference's text
 * round trip: row t = q N + r is (genome1 = genome r, genome2 = genome q) --
 * `mash dist` prints the query as the outer loop -- with
 *   dist[t] = 0 for r == q, else lut32[lut_off[denom] + common] of the pair
 *            (the float32 values the reference's read_csv parses from Mash's
 *            %g text, one table per denominator; denom NULL = s for every pair),
 *   sim[t]  = 1.0f - dist[t] (d_cluster.py:584, IEEE float32),
 *   g1[t] = codes[r], g2[t] = codes[q] (category codes, code_bytes 1, 2 or 4).
 * A pair whose denominator has no table, or whose count exceeds it, fails the
 * call (DREPHIP_ERR_ARG).  sim, g1, g2 nullable.  Host threads (0 = all). */
int drephip_mdb_square(uint32_t N, const uint16_t *common, const uint16_t *denom /* nullable */, uint32_t s,
                       const float *lut32, uint32_t lut_len, const int32_t *lut_off /* s+1 */,
                       const int32_t *codes /* N */, int code_bytes, void *g1, void *g2, float *dist,
                       float *sim, int threads);

/* The pivot of cluster_mash_database (d_cluster.py:620,
 * db.pivot(index="genome1", columns="genome2", values="dist")) on category
 * codes.  drephip_pivot_scan: which of the ncat categories occur in each
 * column (present1/present2), and *period = n when the rows have the layout
 * all_vs_all_MASH returns (codes1 repeating with period n, codes2 constant on
 * each block of n rows), else 0.  A negative code (a missing value) fails with
 * DREPHIP_ERR_UNSUPPORTED (the caller pivots with pandas).
 * drephip_pivot_fill: out[pos1[c1] * n2 + pos2[c2]] = vals of every row
 * (pos: the category's row/column of the pivot, -1 if absent); cells no row
 * names are NaN; two rows naming one cell fail with DREPHIP_ERR_ARG ("Index
 * contains duplicate entries, cannot reshape", pandas' error).  A period from
 * the scan (with n == n1 and nrows == n1 n2) takes the blocked transpose
 * instead of the scatter.  Host threads (0 = all). */
int drephip_pivot_scan(uint64_t nrows, const void *codes1, const void *codes2, int code_bytes, uint32_t ncat,
                       uint8_t *present1, uint8_t *present2, uint64_t *period, int threads);
int drephip_pivot_fill(uint64_t nrows, const void *codes1, const void *codes2, int code_bytes, const int32_t *pos1,
                       const int32_t *pos2, uint32_t ncat, const float *vals, uint32_t n1, uint32_t n2,
                       uint64_t period, float *out, int threads);

/* The sparse path on its own, no context or GPU: the npairs pairs (i[t], j[t])
 * with distance v[t] in [0, 1), each unordered pair at most once; every pair
 * not listed is at 1.0.  Z as scipy.cluster.hierarchy.linkage(squareform(D),
 * method) of that matrix.  DREPHIP_ERR_UNSUPPORTED when the per-component
 * matrices exceed 2^31 cells. */
int drephip_linkage_sparse(uint32_t n, uint64_t npairs, const uint32_t *i, const uint32_t *j, const double *v,
                           int method, double *Z /* (n-1)*4 */);

/* Which path the last drephip_linkage* call on this context took (sparse = 1)
 * and its pair list: pairs below 1.0, components with >= 2 members and the
 * largest one's size (0 for single linkage). */
int drephip_last_linkage_info(drephip_ctx *ctx, int *sparse, uint64_t *pairs, uint32_t *components,
                              uint32_t *largest);

/* Allocates (grow-only, kept in the context) the n x n f64 device matrix the
 * next linkage call of size <= n uses, so that a caller can pay the
 * allocation (80 GB at n = 10^5) outside the clustering step, e.g. before the
 * sketch/all-pairs stages.  Same limits as drephip_linkage. */
int drephip_linkage_reserve(drephip_ctx *ctx, uint32_t n);

/* Step launches of the last linkage call's nearest-neighbour chain that did
 * work (complete / average / weighted on the dense GPU path: ~1.2-1.35 per
 * merge); 0 after the sparse path and for single linkage (Prim). */
int drephip_last_linkage_launches(drephip_ctx *ctx, uint64_t *launches);

/* Host wall-clock split of the last drephip_linkage* call on this context
 * (seconds): the matrix allocation (0 when reserved/reused), the matrix build,
 * the chain (or MST) steps including their setup, the Z readback + scipy's
 * stable sort and relabel, and the whole call. */
int drephip_last_linkage_stats(drephip_ctx *ctx, double *alloc_s, double *matrix_s, double *chain_s,
                               double *finish_s, double *wall_s);

/* HIP-event timing of kernel launches: `kernels` is a bitmask of the kernels
 * to bracket with events (bit w = `which` w of drephip_last_kernel_ms; -1 =
 * all, 0 = none).  Each event pair adds a few microseconds of idle time
 * between dispatches, so a benchmark times only the kernel it reports. */
int drephip_set_timing(drephip_ctx *ctx, int kernels);

/* Per-launch timing of the last sketch/allpairs call on this context
 * (milliseconds, from HIP events on the launch stream): which = 0 sketch hash
 * kernel, 1 sketch finalize kernel, 2 allpairs kernel, 3 table build kernel,
 * 4 the shared-hash screen (grouping + lists, including its host round trips).
 * Returns the count of launches summed into *ms. */
int drephip_last_kernel_ms(drephip_ctx *ctx, int which, double *ms, int *launches);

#ifdef __cplusplus
}
#endif
#endif /* DREPHIP_H */
