/*
 * CPU ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library (oracle/_build/librs_oracle.so).  The product path
 * (shmr_amd, include/shmr_ec.h) never links it and has no CPU fallback.
 *
 * Plain-C restatement of the arithmetic the reference delegates to the
 * third-party crate reed-solomon-erasure 6.0.0 (reference Cargo.toml:16,
 * features=["simd-accel"]; Cargo.lock:1577-1589).  The crate is not vendored
 * and cannot be built here, so its published algorithm is restated:
 *
 *   - field: GF(2^8), polynomial 29 (0x11D), generator 2 (crate build.rs);
 *   - matrix: M = V * inv(V[0..k]), V[r][c] = r^c with 0^0 = 1 (crate core.rs
 *     build_matrix / matrix.rs vandermonde);
 *   - encode: crate code_some_slices loop order -- outer over input shards,
 *     inner over output rows, mul_slice at i == 0 then mul_slice_xor;
 *   - mul_slice on x86_64 with simd-accel: the crate's simd_c/reedsolomon.c
 *     low/high nibble table loop (pshufb), 32 bytes per iteration with AVX2,
 *     scalar MUL_TABLE tail in Rust.  oracle_encode(variant=1) restates it.
 *   - reconstruct: first k present shards in index order, inverse of their
 *     matrix rows, then absent parity re-encoded from the full data.
 *
 * Call sites in the reference: src/vfs/block.rs:405,427 (new/encode in
 * VirtualBlock::sync_data) and block.rs:531,560 (new/reconstruct in
 * VirtualBlock::load_block).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#define FIELD 256
#define POLY 29

static uint8_t LOG_T[FIELD];
static uint8_t EXP_T[FIELD * 2 - 2];
static uint8_t MUL_T[FIELD][FIELD];
static uint8_t MUL_LO[FIELD][16];
static uint8_t MUL_HI[FIELD][16];
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void init_tables(void) {
    unsigned b = 1;
    for (unsigned lg = 0; lg < FIELD - 1; ++lg) {      /* build.rs gen_log_table */
        LOG_T[b] = (uint8_t)lg;
        b <<= 1;
        if (b >= FIELD) b = (b - FIELD) ^ POLY;
    }
    for (unsigned i = 1; i < FIELD; ++i) {              /* build.rs gen_exp_table */
        EXP_T[LOG_T[i]] = (uint8_t)i;
        EXP_T[LOG_T[i] + FIELD - 1] = (uint8_t)i;
    }
    for (unsigned a = 0; a < FIELD; ++a)
        for (unsigned c = 0; c < FIELD; ++c)
            MUL_T[a][c] = (a && c) ? EXP_T[LOG_T[a] + LOG_T[c]] : 0;
    for (unsigned a = 0; a < FIELD; ++a)
        for (unsigned n = 0; n < 16; ++n) {
            MUL_LO[a][n] = MUL_T[a][n];
            MUL_HI[a][n] = MUL_T[a][n << 4];
        }
}
static void tables(void) { pthread_once(&tables_once, init_tables); }

uint8_t oracle_gal_mul(uint8_t a, uint8_t b) { tables(); return MUL_T[a][b]; }
uint8_t oracle_gal_exp(uint8_t a, uint32_t n) {
    tables();
    if (n == 0) return 1;
    if (a == 0) return 0;
    uint32_t lr = (uint32_t)LOG_T[a] * n;
    while (lr >= 255) lr -= 255;
    return EXP_T[lr];
}
static uint8_t gal_div(uint8_t a, uint8_t b) {
    if (a == 0) return 0;
    int lr = (int)LOG_T[a] - (int)LOG_T[b];
    if (lr < 0) lr += 255;
    return EXP_T[lr];
}

/* Gauss-Jordan inverse, n x n, in place on a copy. returns 0 or -1 (singular). */
static int invert(const uint8_t* m, int n, uint8_t* out) {
    uint8_t* w = (uint8_t*)malloc((size_t)n * 2 * n);
    for (int r = 0; r < n; ++r) {
        memcpy(w + (size_t)r * 2 * n, m + (size_t)r * n, n);
        memset(w + (size_t)r * 2 * n + n, 0, n);
        w[(size_t)r * 2 * n + n + r] = 1;
    }
    for (int r = 0; r < n; ++r) {
        uint8_t* rr = w + (size_t)r * 2 * n;
        if (rr[r] == 0) {
            for (int b = r + 1; b < n; ++b) {
                uint8_t* br = w + (size_t)b * 2 * n;
                if (br[r]) {
                    for (int c = 0; c < 2 * n; ++c) { uint8_t t = rr[c]; rr[c] = br[c]; br[c] = t; }
                    break;
                }
            }
        }
        if (rr[r] == 0) { free(w); return -1; }
        if (rr[r] != 1) {
            uint8_t s = gal_div(1, rr[r]);
            for (int c = 0; c < 2 * n; ++c) rr[c] = MUL_T[s][rr[c]];
        }
        for (int o = 0; o < n; ++o) {
            if (o == r) continue;
            uint8_t* orow = w + (size_t)o * 2 * n;
            uint8_t f = orow[r];
            if (f) for (int c = 0; c < 2 * n; ++c) orow[c] ^= MUL_T[f][rr[c]];
        }
    }
    for (int r = 0; r < n; ++r) memcpy(out + (size_t)r * n, w + (size_t)r * 2 * n + n, n);
    free(w);
    return 0;
}

/* out: (k+p) x k row-major. returns 0, or crate error codes (-3/-5/-2). */
int oracle_build_matrix(uint32_t k, uint32_t p, uint8_t* out) {
    tables();
    if (k == 0) return -3;
    if (p == 0) return -5;
    if (k + p > 256) return -2;
    uint32_t t = k + p;
    uint8_t* v = (uint8_t*)malloc((size_t)t * k);
    uint8_t* top_inv = (uint8_t*)malloc((size_t)k * k);
    for (uint32_t r = 0; r < t; ++r)
        for (uint32_t c = 0; c < k; ++c) v[(size_t)r * k + c] = oracle_gal_exp((uint8_t)r, c);
    int rc = invert(v, (int)k, top_inv);
    if (rc == 0) {
        for (uint32_t r = 0; r < t; ++r)
            for (uint32_t c = 0; c < k; ++c) {
                uint8_t acc = 0;
                for (uint32_t i = 0; i < k; ++i) acc ^= MUL_T[v[(size_t)r * k + i]][top_inv[(size_t)i * k + c]];
                out[(size_t)r * k + c] = acc;
            }
    }
    free(v);
    free(top_inv);
    return rc;
}

int oracle_invert(const uint8_t* m, uint32_t n, uint8_t* out) { tables(); return invert(m, (int)n, out); }

/* ---- slice kernels ------------------------------------------------------ */
static void mul_slice_scalar(uint8_t c, const uint8_t* in, uint8_t* out, size_t n, int do_xor) {
    const uint8_t* t = MUL_T[c];
    if (do_xor) for (size_t i = 0; i < n; ++i) out[i] ^= t[in[i]];
    else        for (size_t i = 0; i < n; ++i) out[i] = t[in[i]];
}

#if defined(__x86_64__)
__attribute__((target("avx2")))
static size_t mul_slice_avx2(uint8_t c, const uint8_t* in, uint8_t* out, size_t n, int do_xor) {
    /* simd_c: broadcast the 16-entry low/high nibble tables into both lanes,
     * split each input byte into nibbles, two pshufb lookups, xor. */
    const __m128i lo128 = _mm_loadu_si128((const __m128i*)MUL_LO[c]);
    const __m128i hi128 = _mm_loadu_si128((const __m128i*)MUL_HI[c]);
    const __m256i tlo = _mm256_broadcastsi128_si256(lo128);
    const __m256i thi = _mm256_broadcastsi128_si256(hi128);
    const __m256i mask = _mm256_set1_epi8(0x0f);
    size_t done = 0;
    for (; done + 32 <= n; done += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i*)(in + done));
        __m256i l = _mm256_and_si256(x, mask);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
        __m256i r = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
        if (do_xor) r = _mm256_xor_si256(r, _mm256_loadu_si256((const __m256i*)(out + done)));
        _mm256_storeu_si256((__m256i*)(out + done), r);
    }
    return done;
}
static int have_avx2(void) {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2");
}
#else
static size_t mul_slice_avx2(uint8_t c, const uint8_t* in, uint8_t* out, size_t n, int do_xor) {
    (void)c; (void)in; (void)out; (void)n; (void)do_xor; return 0;
}
static int have_avx2(void) { return 0; }
#endif

static void mul_slice(int variant, uint8_t c, const uint8_t* in, uint8_t* out, size_t n, int do_xor) {
    size_t done = 0;
    if (variant == 1) done = mul_slice_avx2(c, in, out, n, do_xor);
    mul_slice_scalar(c, in + done, out + done, n - done, do_xor);
}

int oracle_has_avx2(void) { return have_avx2(); }

/* rows: nrows x k coefficient matrix (row-major); inputs k slices; outputs nrows. */
static void code_some_slices(int variant, const uint8_t* rows, uint32_t nrows, uint32_t k,
                             const uint8_t* const* in, uint8_t* const* out, size_t len) {
    for (uint32_t i = 0; i < k; ++i)
        for (uint32_t r = 0; r < nrows; ++r)
            mul_slice(variant, rows[(size_t)r * k + i], in[i], out[r], len, i != 0);
}

/* Generic matrix apply: out[r] = XOR_i rows[r][i] (x) in[i]. */
void oracle_apply(int variant, const uint8_t* rows, uint32_t nrows, uint32_t k,
                  const uint8_t* const* in, uint8_t* const* out, size_t len) {
    tables();
    if (variant == 1 && !have_avx2()) variant = 0;
    code_some_slices(variant, rows, nrows, k, in, out, len);
}

/* ReedSolomon::encode for one block; shards[0..k) data, [k..k+p) parity. */
int oracle_encode(int variant, uint32_t k, uint32_t p, uint8_t* const* shards, size_t len) {
    tables();
    if (variant == 1 && !have_avx2()) variant = 0;
    uint8_t* m = (uint8_t*)malloc((size_t)(k + p) * k);
    int rc = oracle_build_matrix(k, p, m);
    if (rc == 0) code_some_slices(variant, m + (size_t)k * k, p, k, (const uint8_t* const*)shards, shards + k, len);
    free(m);
    return rc;
}

/* ReedSolomon::reconstruct{,_data}.  present[i] != 0 marks present shards.
 * Absent shards must point at len-byte buffers; they are filled (absent
 * parity only when !data_only).  returns 0 / -10 (TooFewShardsPresent). */
static int reconstruct_impl(int variant, uint32_t k, uint32_t p, uint8_t* const* shards, const uint8_t* present,
                            size_t len, int data_only);

int oracle_reconstruct(uint32_t k, uint32_t p, uint8_t* const* shards, const uint8_t* present,
                       size_t len, int data_only) {
    tables();
    return reconstruct_impl(0, k, p, shards, present, len, data_only);
}

/* The same with the encode loop's variant (1: the crate's x86 simd_c nibble
 * loop, AVX2): the CPU baseline's reconstruct (tools/ref_cpu_vfs.cpp). */
int oracle_reconstruct_v(int variant, uint32_t k, uint32_t p, uint8_t* const* shards, const uint8_t* present,
                         size_t len, int data_only) {
    tables();
    if (variant == 1 && !have_avx2()) variant = 0;
    return reconstruct_impl(variant, k, p, shards, present, len, data_only);
}

/* The crate's reconstruct (galois_8 ReedSolomon::reconstruct_internal): the
 * first k present shards in index order, decode matrix = inv(M[valid]),
 * absent data rows rebuilt with the SIMD mul_slice loop, absent parity
 * re-encoded from the rebuilt data unless data_only. */
static int reconstruct_impl(int variant, uint32_t k, uint32_t p, uint8_t* const* shards, const uint8_t* present,
                            size_t len, int data_only) {
    uint32_t t = k + p, npresent = 0;
    for (uint32_t i = 0; i < t; ++i) npresent += present[i] ? 1 : 0;
    if (npresent == t) return 0;
    if (npresent < k) return -10;
    uint8_t* m = (uint8_t*)malloc((size_t)t * k);
    oracle_build_matrix(k, p, m);
    uint32_t valid[256], nvalid = 0, inval[256], ninval = 0;
    for (uint32_t i = 0; i < t; ++i) {
        if (present[i]) { if (nvalid < k) valid[nvalid++] = i; }
        else inval[ninval++] = i;
    }
    uint8_t* sub = (uint8_t*)malloc((size_t)k * k);
    uint8_t* dec = (uint8_t*)malloc((size_t)k * k);
    for (uint32_t r = 0; r < k; ++r) memcpy(sub + (size_t)r * k, m + (size_t)valid[r] * k, k);
    int rc = invert(sub, (int)k, dec);
    if (rc == 0) {
        const uint8_t* in[256];
        uint8_t* out[256];
        uint8_t rows[256 * 256];
        uint32_t nr = 0;
        for (uint32_t i = 0; i < k; ++i) in[i] = shards[valid[i]];
        for (uint32_t j = 0; j < ninval; ++j)
            if (inval[j] < k) { memcpy(rows + (size_t)nr * k, dec + (size_t)inval[j] * k, k); out[nr++] = shards[inval[j]]; }
        if (nr) code_some_slices(variant, rows, nr, k, in, out, len);
        if (!data_only) {
            nr = 0;
            for (uint32_t j = 0; j < ninval; ++j)
                if (inval[j] >= k) { memcpy(rows + (size_t)nr * k, m + (size_t)inval[j] * k, k); out[nr++] = shards[inval[j]]; }
            for (uint32_t i = 0; i < k; ++i) in[i] = shards[i];   /* full data after rebuild */
            if (nr) code_some_slices(variant, rows, nr, k, in, out, len);
        }
    }
    free(sub); free(dec); free(m);
    return rc;
}

/* ---- threaded batch encode: one block per task, like rayon into_par_iter
 * over VirtualFile blocks (src/vfs/mod.rs:93-96). ------------------------- */
typedef struct {
    int variant; uint32_t k, p;
    const uint8_t* data; size_t dshard_pitch, dblock_pitch;
    uint8_t* parity; size_t pshard_pitch, pblock_pitch;
    size_t len; const uint8_t* prow;
    size_t nblocks; size_t next; pthread_mutex_t mu;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    const uint8_t* in[256];
    uint8_t* out[256];
    for (;;) {
        pthread_mutex_lock(&j->mu);
        size_t b = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (b >= j->nblocks) break;
        for (uint32_t i = 0; i < j->k; ++i) in[i] = j->data + b * j->dblock_pitch + i * j->dshard_pitch;
        for (uint32_t r = 0; r < j->p; ++r) out[r] = j->parity + b * j->pblock_pitch + r * j->pshard_pitch;
        code_some_slices(j->variant, j->prow, j->p, j->k, in, out, j->len);
    }
    return NULL;
}

/* Encodes nblocks blocks with nthreads threads; returns elapsed seconds of
 * the encode loop alone (the scope of the reference's erasure_encode_duration
 * histogram, block.rs:425-430), or a negative value on error. */
double oracle_encode_batch(int variant, uint32_t k, uint32_t p,
                           const uint8_t* data, size_t dshard_pitch, size_t dblock_pitch,
                           uint8_t* parity, size_t pshard_pitch, size_t pblock_pitch,
                           size_t nblocks, size_t len, int nthreads) {
    tables();
    if (variant == 1 && !have_avx2()) variant = 0;
    uint8_t* m = (uint8_t*)malloc((size_t)(k + p) * k);
    if (oracle_build_matrix(k, p, m) != 0) { free(m); return -1.0; }
    batch_job j = {variant, k, p, data, dshard_pitch, dblock_pitch, parity, pshard_pitch, pblock_pitch,
                   len, m + (size_t)k * k, nblocks, 0, PTHREAD_MUTEX_INITIALIZER};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, batch_worker, &j);
    batch_worker(&j);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(m);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- threaded batch reconstruct (CPU baseline of the decode configs):
 * block b's shard i at base + b * block_pitch + i * shard_pitch, presence
 * flags present[b * (k + p) + i]; one block per task. ---------------------- */
typedef struct {
    int variant; uint32_t k, p;
    uint8_t* base; size_t shard_pitch, block_pitch;
    const uint8_t* present; size_t len; int data_only;
    size_t nblocks; size_t next; int rc; pthread_mutex_t mu;
} rbatch_job;

static void* rbatch_worker(void* arg) {
    rbatch_job* j = (rbatch_job*)arg;
    uint8_t* sh[256];
    const uint32_t t = j->k + j->p;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        size_t b = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (b >= j->nblocks) break;
        for (uint32_t i = 0; i < t; ++i) sh[i] = j->base + b * j->block_pitch + i * j->shard_pitch;
        int rc = reconstruct_impl(j->variant, j->k, j->p, sh, j->present + b * t, j->len, j->data_only);
        if (rc) { pthread_mutex_lock(&j->mu); j->rc = rc; pthread_mutex_unlock(&j->mu); }
    }
    return NULL;
}

double oracle_reconstruct_batch(int variant, uint32_t k, uint32_t p, uint8_t* base, size_t shard_pitch,
                                size_t block_pitch, const uint8_t* present, size_t nblocks, size_t len,
                                int data_only, int nthreads) {
    tables();
    if (variant == 1 && !have_avx2()) variant = 0;
    rbatch_job j = {variant, k, p, base, shard_pitch, block_pitch, present, len, data_only, nblocks, 0, 0,
                    PTHREAD_MUTEX_INITIALIZER};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, rbatch_worker, &j);
    rbatch_worker(&j);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (j.rc) return -1.0;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- threaded VirtualBlock::sync_data Erasure arm minus disk I/O
 * (block.rs:406-430): per block, chunks(S).to_vec() of the size-byte buffer,
 * the last chunk resized to S, p + (k - nchunks) zero shards appended, then
 * encode; the Vec allocations are part of the timed work, as in the
 * reference.  Parity is written to parity + b * p * S for checking. -------- */
typedef struct {
    int variant; uint32_t k, p;
    const uint8_t* src; size_t size, S;
    uint8_t* parity; const uint8_t* prow;
    size_t nblocks; size_t next; pthread_mutex_t mu;
} sbatch_job;

static void* sbatch_worker(void* arg) {
    sbatch_job* j = (sbatch_job*)arg;
    uint8_t* sh[256];
    for (;;) {
        pthread_mutex_lock(&j->mu);
        size_t b = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (b >= j->nblocks) break;
        const uint8_t* buf = j->src + b * j->size;
        const size_t nchunks = (j->size + j->S - 1) / j->S;
        const uint32_t t = j->k + j->p;
        for (uint32_t i = 0; i < t; ++i) {
            sh[i] = (uint8_t*)malloc(j->S);
            if (i < nchunks) {
                const size_t off = (size_t)i * j->S;
                const size_t n = off + j->S <= j->size ? j->S : j->size - off;
                memcpy(sh[i], buf + off, n);
                if (n < j->S) memset(sh[i] + n, 0, j->S - n);
            } else {
                memset(sh[i], 0, j->S);
            }
        }
        code_some_slices(j->variant, j->prow, j->p, j->k, (const uint8_t* const*)sh, sh + j->k, j->S);
        for (uint32_t r = 0; r < j->p; ++r) memcpy(j->parity + (b * j->p + r) * j->S, sh[j->k + r], j->S);
        for (uint32_t i = 0; i < t; ++i) free(sh[i]);
    }
    return NULL;
}

double oracle_sync_data_batch(int variant, uint32_t k, uint32_t p, const uint8_t* src, size_t size, size_t S,
                              uint8_t* parity, size_t nblocks, int nthreads) {
    tables();
    if (variant == 1 && !have_avx2()) variant = 0;
    if (S == 0 || (size + S - 1) / S > k) return -1.0;
    uint8_t* m = (uint8_t*)malloc((size_t)(k + p) * k);
    if (oracle_build_matrix(k, p, m) != 0) { free(m); return -1.0; }
    sbatch_job j = {variant, k, p, src, size, S, parity, m + (size_t)k * k, nblocks, 0, PTHREAD_MUTEX_INITIALIZER};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, sbatch_worker, &j);
    sbatch_worker(&j);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(m);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
