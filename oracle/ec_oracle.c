/*
 * ec_oracle.c -- CPU restatement of the reference's GF(2^8) Reed-Solomon path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the "port"
 * CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (erasure_coding_test_amd/,
 * libecgpu.so, libjerasure_amd.so) never links, loads or calls it.
 *
 * Pinning: restated from the reference (canghaiyang/Erasure_Coding_Test, the
 * vendored Jerasure 1.2 under src/erasure_coding/) and checked bit-for-bit
 * against (a) the reference compiled from its own sources by oracle/Makefile
 * into oracle/_ref/ and (b) golden vectors generated from that build
 * (tests/golden/, script tests/golden/make_golden.py).
 *
 * Only w = 8 is restated (the north-star path).  Byte semantics differ from
 * the reference in one documented way: the reference's 8-byte add/XOR loops
 * over-run regions whose size is not a multiple of 8
 * (galois.cpp:452-465, :748-753); this restatement is exact on [0, size)
 * and writes nothing beyond it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define GF_POLY 0x11D /* prim_poly[8] = 0435, galois.cpp:57 */

static int g_log[256];           /* galois_log_tables[8]               */
static int g_ilog_store[255 * 3]; /* ilog replicated 3x, galois.cpp:185-189 */
static const int *g_ilog;        /* = g_ilog_store + 255               */
static uint8_t g_mul[256][256];  /* galois_mult_tables[8], row = multiplicand */
static int g_div[256][256];      /* galois_div_tables[8]               */

/* galois_create_log_tables(8), galois.cpp:152-191 */
static void build_log_tables(void) {
  for (int j = 0; j < 256; j++) g_log[j] = 255;
  for (int j = 0; j < 255 * 3; j++) g_ilog_store[j] = 0;
  int b = 1;
  for (int j = 0; j < 255; j++) {
    g_log[b] = j;
    g_ilog_store[j] = b;
    b <<= 1;
    if (b & 0x100) b = (b ^ GF_POLY) & 0xFF;
  }
  for (int j = 0; j < 255; j++) {
    g_ilog_store[j + 255] = g_ilog_store[j];
    g_ilog_store[j + 510] = g_ilog_store[j];
  }
  g_ilog = g_ilog_store + 255;
}

/* galois_create_mult_tables(8), galois.cpp:218-267 */
__attribute__((constructor)) static void orc_init(void) {
  build_log_tables();
  for (int x = 0; x < 256; x++) {
    for (int y = 0; y < 256; y++) {
      if (x == 0 || y == 0) {
        g_mul[x][y] = 0;
        g_div[x][y] = (y == 0) ? -1 : 0;
      } else {
        g_mul[x][y] = (uint8_t)g_ilog[g_log[x] + g_log[y]];
        g_div[x][y] = g_ilog[g_log[x] - g_log[y]];
      }
    }
  }
}

/* ---- scalar field ops: galois.cpp:322-360, :367-398, :597-603, :269-289 -- */
int orc_gf_mul(int a, int b) { return g_mul[a & 0xFF][b & 0xFF]; }
int orc_gf_div(int a, int b) { return g_div[a & 0xFF][b & 0xFF]; }
int orc_gf_inverse(int y) { return (y == 0) ? -1 : g_div[1][y & 0xFF]; }
int orc_gf_log(int v) { return g_log[v & 0xFF]; }
int orc_gf_ilog(int v) { return (v >= -255 && v < 510) ? g_ilog[v] : -1; }

/* ---- Vandermonde: reed_sol.cpp:227-255 (extended), :257-352 (distribution),
 *      :63-84 (coding part).  Returns 0, or -1 where the reference returns NULL. */
static int extended_vandermonde(int rows, int cols, int *vdm) {
  if (256 < rows || 256 < cols) return -1;          /* reed_sol.cpp:232-233 */
  for (int i = 0; i < rows * cols; i++) vdm[i] = 0;
  vdm[0] = 1;                                       /* row 0 = e0       */
  if (rows == 1) return 0;
  vdm[(rows - 1) * cols + cols - 1] = 1;            /* last row = e_{cols-1} */
  if (rows == 2) return 0;
  for (int i = 1; i < rows - 1; i++) {              /* row i = powers of i */
    int p = 1;
    for (int j = 0; j < cols; j++) {
      vdm[i * cols + j] = p;
      p = orc_gf_mul(p, i);
    }
  }
  return 0;
}

static int big_vandermonde_distribution(int rows, int cols, int *d) {
  if (cols >= rows) return -1;                      /* reed_sol.cpp:263 */
  if (extended_vandermonde(rows, cols, d) < 0) return -1;
  for (int i = 1; i < cols; i++) {
    /* find a row r >= i with d[r][i] != 0 and swap it into row i (:273-289) */
    int r = i;
    while (r < rows && d[r * cols + i] == 0) r++;
    if (r >= rows) return -1; /* reference exits here (:275-279) */
    if (r != i)
      for (int c = 0; c < cols; c++) {
        int t = d[r * cols + c];
        d[r * cols + c] = d[i * cols + c];
        d[i * cols + c] = t;
      }
    /* scale column i so d[i][i] == 1 (:293-300) */
    if (d[i * cols + i] != 1) {
      int inv = orc_gf_div(1, d[i * cols + i]);
      for (int rr = 0; rr < rows; rr++) d[rr * cols + i] = orc_gf_mul(inv, d[rr * cols + i]);
    }
    /* clear row i off the diagonal with column operations (:308-319) */
    for (int j = 0; j < cols; j++) {
      int e = d[i * cols + j];
      if (j != i && e != 0)
        for (int rr = 0; rr < rows; rr++)
          d[rr * cols + j] ^= orc_gf_mul(e, d[rr * cols + i]);
    }
  }
  /* row `cols` becomes all ones by scaling columns over the coding rows (:324-336) */
  for (int j = 0; j < cols; j++) {
    int e = d[cols * cols + j];
    if (e != 1) {
      int inv = orc_gf_div(1, e);
      for (int rr = cols; rr < rows; rr++) d[rr * cols + j] = orc_gf_mul(inv, d[rr * cols + j]);
    }
  }
  /* column 0 of the remaining coding rows becomes one by row scaling (:341-349) */
  for (int rr = cols + 1; rr < rows; rr++) {
    int e = d[rr * cols];
    if (e != 1) {
      int inv = orc_gf_div(1, e);
      for (int j = 0; j < cols; j++) d[rr * cols + j] = orc_gf_mul(d[rr * cols + j], inv);
    }
  }
  return 0;
}

int orc_vandermonde_coding_matrix(int k, int m, int *out /* m*k */) {
  int *d = (int *)malloc(sizeof(int) * (size_t)(k + m) * k);
  if (!d) return -1;
  int rc = big_vandermonde_distribution(k + m, k, d);
  if (rc == 0) memcpy(out, d + k * k, sizeof(int) * (size_t)m * k);
  free(d);
  return rc;
}

/* ---- GF Gauss-Jordan inversion, jerasure.cpp:360-445 (destroys mat) ---- */
int orc_invert_matrix(int *mat, int *inv, int n) {
  for (int i = 0; i < n * n; i++) inv[i] = 0;
  for (int i = 0; i < n; i++) inv[i * n + i] = 1;
  for (int i = 0; i < n; i++) {
    if (mat[i * n + i] == 0) {
      int r = i + 1;
      while (r < n && mat[r * n + i] == 0) r++;
      if (r == n) return -1;
      for (int c = 0; c < n; c++) {
        int t = mat[i * n + c]; mat[i * n + c] = mat[r * n + c]; mat[r * n + c] = t;
        t = inv[i * n + c]; inv[i * n + c] = inv[r * n + c]; inv[r * n + c] = t;
      }
    }
    int p = mat[i * n + i];
    if (p != 1) {
      int s = orc_gf_div(1, p);
      for (int c = 0; c < n; c++) {
        mat[i * n + c] = orc_gf_mul(mat[i * n + c], s);
        inv[i * n + c] = orc_gf_mul(inv[i * n + c], s);
      }
    }
    for (int r = i + 1; r < n; r++) {
      int e = mat[r * n + i];
      if (e == 0) continue;
      for (int c = 0; c < n; c++) {
        mat[r * n + c] ^= orc_gf_mul(e, mat[i * n + c]);
        inv[r * n + c] ^= orc_gf_mul(e, inv[i * n + c]);
      }
    }
  }
  for (int i = n - 1; i >= 0; i--)
    for (int r = 0; r < i; r++) {
      int e = mat[r * n + i];
      if (e == 0) continue;
      mat[r * n + i] = 0;
      for (int c = 0; c < n; c++) inv[r * n + c] ^= orc_gf_mul(e, inv[i * n + c]);
    }
  return 0;
}

/* ---- jerasure_erasures_to_erased, jerasure.cpp:507-532 ----
 * Fills erased[k+m]; returns 0, or -1 where the reference returns NULL. */
int orc_erasures_to_erased(int k, int m, const int *erasures, int *erased) {
  int alive = k + m;
  for (int i = 0; i < k + m; i++) erased[i] = 0;
  for (int i = 0; erasures[i] != -1; i++) {
    if (!erased[erasures[i]]) {
      erased[erasures[i]] = 1;
      if (--alive < k) return -1;
    }
  }
  return 0;
}

/* ---- jerasure_make_decoding_matrix, jerasure.cpp:84-112 ---- */
int orc_make_decoding_matrix(int k, int m, const int *matrix, const int *erased, int *dm, int *dm_ids) {
  (void)m;
  for (int i = 0, j = 0; j < k; i++)
    if (!erased[i]) dm_ids[j++] = i;
  int *t = (int *)malloc(sizeof(int) * (size_t)k * k);
  if (!t) return -1;
  for (int i = 0; i < k; i++) {
    if (dm_ids[i] < k) {
      for (int j = 0; j < k; j++) t[i * k + j] = (j == dm_ids[i]);
    } else {
      memcpy(t + i * k, matrix + (dm_ids[i] - k) * k, sizeof(int) * (size_t)k);
    }
  }
  int rc = orc_invert_matrix(t, dm, k);
  free(t);
  return rc;
}

/* ---- region primitives ----
 * galois_w08_region_multiply, galois.cpp:415-467.  add=0 (or r2 NULL):
 * bytewise dst = c*src.  add=1: eight products are packed into one 64-bit
 * word and XORed into dst (galois.cpp:452-465); same here for whole words,
 * exact bytewise for the tail. */
void orc_region_multiply(const uint8_t *src, int c, long n, uint8_t *r2, int add) {
  uint8_t *dst = r2 ? r2 : (uint8_t *)src;
  const uint8_t *row = g_mul[c & 0xFF];
  if (r2 == NULL || !add) {
    for (long i = 0; i < n; i++) dst[i] = row[src[i]];
    return;
  }
  long i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t p = 0, d;
    for (int j = 0; j < 8; j++) p |= (uint64_t)row[src[i + j]] << (8 * j);
    memcpy(&d, dst + i, 8);
    d ^= p;
    memcpy(dst + i, &d, 8);
  }
  for (; i < n; i++) dst[i] ^= row[src[i]];
}

/* galois_region_xor, galois.cpp:731-754: r3 = r1 ^ r2, word-wise + exact tail */
void orc_region_xor(const uint8_t *r1, const uint8_t *r2, uint8_t *r3, long n) {
  long i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t a, b;
    memcpy(&a, r1 + i, 8);
    memcpy(&b, r2 + i, 8);
    a ^= b;
    memcpy(r3 + i, &a, 8);
  }
  for (; i < n; i++) r3[i] = r1[i] ^ r2[i];
}

/* ---- jerasure_matrix_dotprod, jerasure.cpp:561-620 (w = 8) ----
 * Unit coefficients first (memcpy then XOR), then the others via the
 * region multiply with add = "already initialised".  All-zero rows leave
 * the destination untouched. */
static uint8_t *pick(int id, int k, uint8_t **data, uint8_t **coding) {
  return id < k ? data[id] : coding[id - k];
}

void orc_matrix_dotprod(int k, const int *row, const int *src_ids, int dest_id,
                        uint8_t **data, uint8_t **coding, long size) {
  uint8_t *dst = pick(dest_id, k, data, coding);
  int init = 0;
  for (int i = 0; i < k; i++) {
    if (row[i] != 1) continue;
    uint8_t *s = src_ids ? pick(src_ids[i], k, data, coding) : data[i];
    if (!init) { memcpy(dst, s, (size_t)size); init = 1; }
    else orc_region_xor(s, dst, dst, size);
  }
  for (int i = 0; i < k; i++) {
    if (row[i] == 0 || row[i] == 1) continue;
    uint8_t *s = src_ids ? pick(src_ids[i], k, data, coding) : data[i];
    orc_region_multiply(s, row[i], size, dst, init);
    init = 1;
  }
}

/* jerasure_matrix_encode, jerasure.cpp:285-299 */
void orc_matrix_encode(int k, int m, const int *matrix, uint8_t **data, uint8_t **coding, long size) {
  for (int i = 0; i < m; i++) orc_matrix_dotprod(k, matrix + i * k, NULL, k + i, data, coding, size);
}

/* jerasure_matrix_decode, jerasure.cpp:153-254 (w = 8).  Returns 0 / -1. */
int orc_matrix_decode(int k, int m, const int *matrix, int row_k_ones, const int *erasures,
                      uint8_t **data, uint8_t **coding, long size) {
  int *erased = (int *)malloc(sizeof(int) * (size_t)(k + m));
  if (!erased) return -1;
  if (orc_erasures_to_erased(k, m, erasures, erased) < 0) { free(erased); return -1; }
  int edd = 0, lastdrive = k;
  for (int i = 0; i < k; i++)
    if (erased[i]) { edd++; lastdrive = i; }
  if (!row_k_ones || erased[k]) lastdrive = k;

  int *dm_ids = NULL, *dm = NULL;
  if (edd > 1 || (edd > 0 && (!row_k_ones || erased[k]))) {
    dm_ids = (int *)malloc(sizeof(int) * (size_t)k);
    dm = (int *)malloc(sizeof(int) * (size_t)k * k);
    if (!dm_ids || !dm || orc_make_decoding_matrix(k, m, matrix, erased, dm, dm_ids) < 0) {
      free(erased); free(dm_ids); free(dm);
      return -1;
    }
  }
  for (int i = 0; edd > 0 && i < lastdrive; i++) {
    if (!erased[i]) continue;
    orc_matrix_dotprod(k, dm + i * k, dm_ids, i, data, coding, size);
    edd--;
  }
  if (edd > 0) { /* row_k_ones shortcut, jerasure.cpp:232-239 */
    int *tmpids = (int *)malloc(sizeof(int) * (size_t)k);
    for (int i = 0; i < k; i++) tmpids[i] = (i < lastdrive) ? i : i + 1;
    orc_matrix_dotprod(k, matrix, tmpids, lastdrive, data, coding, size);
    free(tmpids);
  }
  for (int i = 0; i < m; i++)
    if (erased[k + i]) orc_matrix_dotprod(k, matrix + i * k, NULL, i + k, data, coding, size);
  free(erased); free(dm_ids); free(dm);
  return 0;
}

/* ---- multi-threaded encode: byte-range split like encode_mul_thread,
 *      client_main.cpp:1074-1164 (thread 0 takes the remainder). ---- */
typedef struct {
  int k, m;
  const int *matrix;
  uint8_t *data[256], *coding[256];
  long size;
} orc_job;

static void *orc_job_run(void *arg) {
  orc_job *j = (orc_job *)arg;
  orc_matrix_encode(j->k, j->m, j->matrix, j->data, j->coding, j->size);
  return NULL;
}

int orc_matrix_encode_mt(int k, int m, const int *matrix, uint8_t **data, uint8_t **coding,
                         long size, int nthreads) {
  if (nthreads < 1 || nthreads > 256 || k > 256 || m > 256) return -1;
  orc_job *jobs = (orc_job *)calloc((size_t)nthreads, sizeof(orc_job));
  pthread_t *tid = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  long off = 0;
  for (int t = 0; t < nthreads; t++) {
    long len = size / nthreads + (t == 0 ? size % nthreads : 0);
    jobs[t].k = k; jobs[t].m = m; jobs[t].matrix = matrix; jobs[t].size = len;
    for (int i = 0; i < k; i++) jobs[t].data[i] = data[i] + off;
    for (int i = 0; i < m; i++) jobs[t].coding[i] = coding[i] + off;
    off += len;
    pthread_create(&tid[t], NULL, orc_job_run, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(tid[t], NULL);
  free(jobs); free(tid);
  return 0;
}

/* ---- deterministic synthetic shards and digests ---- */
static uint64_t splitmix64_next(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

void orc_splitmix_fill(uint8_t *buf, long n, uint64_t seed) {
  uint64_t s = seed;
  long i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v = splitmix64_next(&s);
    memcpy(buf + i, &v, 8);
  }
  if (i < n) {
    uint64_t v = splitmix64_next(&s);
    memcpy(buf + i, &v, (size_t)(n - i));
  }
}

uint64_t orc_fnv1a64(const uint8_t *buf, long n) {
  uint64_t h = 0xCBF29CE484222325ULL;
  for (long i = 0; i < n; i++) { h ^= buf[i]; h *= 0x100000001B3ULL; }
  return h;
}
