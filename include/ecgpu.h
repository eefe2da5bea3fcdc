/*
 * ecgpu.h -- C ABI of the MI355X (gfx950) Reed-Solomon GF(2^8) coding library.
 *
 * The drop-in boundary of this repo.  Every entry point is extern "C", takes
 * plain pointers and sizes, and replaces one function of the reference's
 * coding surface (canghaiyang/Erasure_Coding_Test, vendored Jerasure 1.2:
 * include/galois.h, include/jerasure.h, include/reed_sol.h).  The cited
 * file:line is the reference function each entry point replaces; argument
 * meaning, ownership (malloc'd results freed with free()) and return
 * conventions are the reference's.  libjerasure_amd.so re-exports the same
 * functions under the reference's own (C++-mangled) names, so callers built
 * against the reference headers link unchanged.
 *
 * Hot path (GPU): ecgpu_jerasure_matrix_encode / _decode / _dotprod,
 * ecgpu_galois_w08_region_multiply, ecgpu_galois_region_xor,
 * ecgpu_jerasure_do_parity, ecgpu_reed_sol_r6_encode and the batched
 * device-resident plan API below.  The matrix calls take w = 8 (the north
 * star), 16 or 32 (wide-word kernels; size a whole number of w/8-byte words,
 * else ECGPU_ERR_ARG) and so do the w16/w32 region functions.  These accept host OR device pointers
 * (classified per buffer; host buffers are staged through HBM) and are
 * synchronous: results are valid on return, like the reference.  A call
 * whose buffers are all host memory and that moves fewer than
 * ECGPU_MIN_OFFLOAD_KIB bytes (distinct buffers x size; by default the
 * measured crossover for the host's SIMD level, 16 MiB with GFNI,
 * ecgpu_min_offload_bytes; every such call with ECGPU_GPU=0)
 * runs on the library's own CPU executor, where the GPU round trip would
 * cost more (counted by ecgpu_cpu_call_count).  A HIP failure on
 * a call whose buffers are all host memory, before it overwrote one of its
 * sources, completes on the CPU (no new failure modes; counted
 * by ecgpu_fallback_count, the first one logged on stderr) unless the
 * ECGPU_CPU_FALLBACK knob is 0; any other HIP failure returns ECGPU_ERR_HIP
 * (through the void-returning drop-in names: exits with a message).  The
 * Python package turns the fallback off and the threshold to 0 unless the
 * environment sets them, and the bench and tests assert both counts are 0.
 * Buffers of one
 * call are identical or disjoint: a written region that partially overlaps
 * another region of the call returns ECGPU_ERR_ARG before anything runs
 * (see ecgpu_plan_check_buffers).
 *
 * Host-only (no GPU touched): field arithmetic, matrix construction,
 * inversion and decode planning.
 */
#ifndef ECGPU_H
#define ECGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define ECGPU_API __attribute__((visibility("default")))
#else
#define ECGPU_API
#endif

enum {
  ECGPU_OK = 0,
  ECGPU_ERR = -1,         /* reference-style failure (e.g. too many erasures) */
  ECGPU_ERR_ARG = -2,     /* invalid argument (w, k, m, size, pointers)       */
  ECGPU_ERR_HIP = -3,     /* HIP runtime / kernel launch failure              */
  ECGPU_ERR_NOMEM = -4
};

enum { ECGPU_KERNEL_PERM = 0, ECGPU_KERNEL_LDS = 1 };

/* ---------------------------------------------------------------- misc -- */
ECGPU_API const char* ecgpu_version(void);
/* Content IDs of the built library (16 hex digits): what = 0 the whole
 * library, 1 the w = 8 kernels and their dispatch (the identity a rocprofv3
 * PMC record of the bench's launches is valid for), 2 the w = 16 / 32
 * kernels, 3 the GF(2) packet kernels. */
ECGPU_API const char* ecgpu_build_id(int what);
ECGPU_API const char* ecgpu_last_error(void);         /* thread-local message */
/* Tuning / A-B switches (knobs.hpp lists them: the residency cap, engines,
 * store policy, wide-word forms, staging thresholds, shard skew).  Each is
 * read once from its ECGPU_* environment variable at first use; set_knob
 * overrides it for the whole process (name = "ECGPU_CAP" or "cap"), reset_knob
 * restores the environment's value (NULL: every knob).  ECGPU_ERR_ARG for an
 * unknown name.  Plans take the engine / store-policy knobs when created. */
ECGPU_API int ecgpu_set_knob(const char* name, int value);
ECGPU_API int ecgpu_reset_knob(const char* name);
ECGPU_API int ecgpu_get_knob(const char* name, int* value);
ECGPU_API void ecgpu_free(void* p);                    /* == free()           */
/* SURVEY §8b failure contract: synchronous calls completed on the CPU after a
 * HIP error (process total), and whether a sticky HIP error (kernel fault,
 * lost device) marked `device` unusable -- with ECGPU_CPU_FALLBACK on, later
 * host-memory calls on it run on the CPU without touching it. */
ECGPU_API int64_t ecgpu_fallback_count(void);
ECGPU_API int ecgpu_device_lost(int device);
/* Synchronous host-memory calls run on the CPU executor by choice: below
 * ECGPU_MIN_OFFLOAD_KIB, or with ECGPU_GPU=0 (process total). */
ECGPU_API int64_t ecgpu_cpu_call_count(void);
/* The bytes-moved threshold in force (0: every call to the GPU): the
 * ECGPU_MIN_OFFLOAD_KIB knob when set, else by the executor's SIMD level --
 * 16 MiB with AVX-512 + GFNI, 4 MiB with AVX2, 256 KiB scalar, each the
 * measured crossover on the MI355X host. */
ECGPU_API int64_t ecgpu_min_offload_bytes(void);
/* The devices synchronous host-memory calls spread over (default: unset, the
 * caller's current device).  Each calling thread is given one entry,
 * round-robin in the order threads make their first such call, and keeps it,
 * so concurrent callers (the reference client's byte-range encode pthreads,
 * client_main.cpp:1074-1164) each drive their own GPU.  Also read from
 * ECGPU_DEVICES ("all" or "0,1,2,..."; repeats allowed) at first use; n = 0
 * unsets.  A list naming a device HIP does not show this process is
 * rejected (ECGPU_ERR_ARG; the environment's list is ignored with one stderr
 * line), so a typo cannot send every call to the CPU fallback.  A forced
 * ECGPU_DEVICE wins; calls naming device memory run on the
 * current device.  get_devices returns the list's length (0 if unset) and
 * copies up to cap entries; call_device is the device this thread's next
 * host-memory call runs on. */
ECGPU_API int ecgpu_set_devices(int n, const int* devices);
ECGPU_API int ecgpu_get_devices(int* out, int cap);
ECGPU_API int ecgpu_call_device(void);
/* Specialised w = 8 column launches so far per engine (kind =
 * ECGPU_KERNEL_PERM / ECGPU_KERNEL_LDS): which engine a knob setting reached. */
ECGPU_API int64_t ecgpu_engine_launches(int kind);

/* ------------------------------------- GF(2^w) scalar ops (host only) --- */
ECGPU_API int ecgpu_galois_single_multiply(int a, int b, int w); /* galois.cpp:322-360 */
ECGPU_API int ecgpu_galois_single_divide(int a, int b, int w);   /* galois.cpp:367-398 */
ECGPU_API int ecgpu_galois_inverse(int a, int w);                /* galois.cpp:597-603 */
/* log: value in [0, 2^w); ilog: value in [-(2^w - 1), 2(2^w - 1)).  -1 for a
 * value outside the table or w > 30 (the reference reads out of bounds / exits) */
ECGPU_API int ecgpu_galois_log(int value, int w);                /* galois.cpp:280-289 */
ECGPU_API int ecgpu_galois_ilog(int value, int w);               /* galois.cpp:269-278 */
/* Field tables, built once per w and kept for the library's lifetime
 * (galois.cpp:627-665, galois.h:46-66): 0 / -1 like galois_create_*_tables, NULL where the
 * reference cannot build them.  mult / div: 2^(2w) entries indexed (x << w) | y
 * (w <= 13); log: 2^w entries; ilog: offset pointer valid on
 * [-(2^w - 1), 2(2^w - 1)) (w <= 30). */
ECGPU_API int ecgpu_galois_create_log_tables(int w);             /* galois.cpp:152-191 */
ECGPU_API int ecgpu_galois_create_mult_tables(int w);            /* galois.cpp:218-267 */
ECGPU_API int* ecgpu_galois_get_mult_table(int w);
ECGPU_API int* ecgpu_galois_get_div_table(int w);
ECGPU_API int* ecgpu_galois_get_log_table(int w);
ECGPU_API int* ecgpu_galois_get_ilog_table(int w);
ECGPU_API int ecgpu_galois_shift_multiply(int a, int b, int w);  /* galois.cpp:292-320 */
ECGPU_API int ecgpu_galois_shift_inverse(int a, int w);          /* galois.cpp:605-625 */
/* The w = 32 split tables: 0 (or -1 if they cannot be allocated), and the
 * product read from them (galois.cpp:756-789, :791-809). */
ECGPU_API int ecgpu_galois_create_split_w8_tables(void);
ECGPU_API int ecgpu_galois_split_w8_multiply(int x, int y);

/* ------------------------------------------- matrices (host only) ------- */
ECGPU_API int* ecgpu_reed_sol_vandermonde_coding_matrix(int k, int m, int w);            /* reed_sol.cpp:63-84   */
ECGPU_API int* ecgpu_reed_sol_extended_vandermonde_matrix(int rows, int cols, int w);    /* reed_sol.cpp:227-255 */
ECGPU_API int* ecgpu_reed_sol_big_vandermonde_distribution_matrix(int rows, int cols, int w); /* reed_sol.cpp:257-352 */
ECGPU_API int* ecgpu_reed_sol_r6_coding_matrix(int k, int w);                            /* reed_sol.cpp:43-61   */
ECGPU_API int ecgpu_jerasure_invert_matrix(int* mat, int* inv, int rows, int w);         /* jerasure.cpp:360-445 */
ECGPU_API int ecgpu_jerasure_invertible_matrix(int* mat, int rows, int w);               /* jerasure.cpp:447-502 */
ECGPU_API int* ecgpu_jerasure_matrix_multiply(int* m1, int* m2, int r1, int c1, int r2, int c2, int w); /* jerasure.cpp:1126-1141 */
ECGPU_API int* ecgpu_jerasure_erasures_to_erased(int k, int m, int* erasures);           /* jerasure.cpp:507-532 */
ECGPU_API int ecgpu_jerasure_make_decoding_matrix(int k, int m, int w, int* matrix, int* erased,
                                                  int* decoding_matrix, int* dm_ids);    /* jerasure.cpp:84-112  */
ECGPU_API int* ecgpu_jerasure_matrix_to_bitmatrix(int k, int m, int w, int* matrix);      /* jerasure.cpp:257-283 */
ECGPU_API int ecgpu_jerasure_make_decoding_bitmatrix(int k, int m, int w, int* matrix, int* erased,
                                                     int* decoding_matrix, int* dm_ids); /* jerasure.cpp:115-151 */
ECGPU_API int ecgpu_jerasure_invert_bitmatrix(int* mat, int* inv, int rows);              /* jerasure.cpp:1034-1089 */
ECGPU_API int ecgpu_jerasure_invertible_bitmatrix(int* mat, int rows);                    /* jerasure.cpp:1091-1124 */

/* Fused decode plan (host only): the single linear map that
 * jerasure_matrix_decode (jerasure.cpp:153-254) applies, over shard ids
 * 0..k+m-1.  On return out_ids[0..*n_out) are the shard ids written,
 * src_ids[0..*n_src) the shard ids read, coefs row-major n_out x n_src.
 * Arrays must hold k+m (ids) and (k+m)^2 (coefs) entries.  Returns 0 or -1
 * exactly where the reference decode returns -1.  w = 8, 16 or 32. */
ECGPU_API int ecgpu_decode_plan(int k, int m, int w, const int* matrix, int row_k_ones, const int* erasures,
                                int* out_ids, int* n_out, int* src_ids, int* n_src, int* coefs);

/* ------------------------------------ hot path: reference semantics ----- */
/* jerasure.cpp:285-299.  w = 8, 16 or 32. */
ECGPU_API int ecgpu_jerasure_matrix_encode(int k, int m, int w, int* matrix, char** data_ptrs, char** coding_ptrs,
                                           int size);
/* jerasure.cpp:153-254.  Returns 0 / -1 like the reference. */
ECGPU_API int ecgpu_jerasure_matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures,
                                           char** data_ptrs, char** coding_ptrs, int size);
/* jerasure.cpp:561-620.  w = 1, 8, 16 or 32 (w = 1: the XOR of the sources
 * whose coefficient is 1, as in the reference, which has no w = 1 multiply). */
ECGPU_API int ecgpu_jerasure_matrix_dotprod(int k, int w, int* matrix_row, int* src_ids, int dest_id,
                                            char** data_ptrs, char** coding_ptrs, int size);
/* jerasure.cpp:347-358 */
ECGPU_API int ecgpu_jerasure_do_parity(int k, char** data_ptrs, char* parity_ptr, int size);
/* galois.cpp:415-467 */
ECGPU_API int ecgpu_galois_w08_region_multiply(char* region, int multby, int nbytes, char* r2, int add);
/* galois.cpp:731-754 */
ECGPU_API int ecgpu_galois_region_xor(char* r1, char* r2, char* r3, int nbytes);
/* galois.cpp:469-542 (nbytes/2 words) and galois.cpp:666-727 (nbytes/4 words) */
ECGPU_API int ecgpu_galois_w16_region_multiply(char* region, int multby, int nbytes, char* r2, int add);
ECGPU_API int ecgpu_galois_w32_region_multiply(char* region, int multby, int nbytes, char* r2, int add);
/* reed_sol.cpp:200-225 (returns 1; 0 for w other than 8/16/32) and the
 * multiply-by-2 helpers reed_sol.cpp:112-152, :158-198, :90-106 */
ECGPU_API int ecgpu_reed_sol_r6_encode(int k, int w, char** data_ptrs, char** coding_ptrs, int size);
ECGPU_API int ecgpu_reed_sol_galois_w08_region_multby_2(char* region, int nbytes);
ECGPU_API int ecgpu_reed_sol_galois_w16_region_multby_2(char* region, int nbytes);
ECGPU_API int ecgpu_reed_sol_galois_w32_region_multby_2(char* region, int nbytes);
/* GF(2) packet coding on the GPU: a device is w packets of packetsize bytes
 * per super-packet (size % (w*packetsize) must be 0, else ECGPU_ERR_ARG).
 * jerasure.cpp:301-345, :1346-1363, :623-703 (0 / -1 like the reference). */
ECGPU_API int ecgpu_jerasure_bitmatrix_dotprod(int k, int w, int* bitmatrix_row, int* src_ids, int dest_id,
                                               char** data_ptrs, char** coding_ptrs, int size, int packetsize);
ECGPU_API int ecgpu_jerasure_bitmatrix_encode(int k, int m, int w, int* bitmatrix, char** data_ptrs,
                                              char** coding_ptrs, int size, int packetsize);
ECGPU_API int ecgpu_jerasure_bitmatrix_decode(int k, int m, int w, int* bitmatrix, int row_k_ones, int* erasures,
                                              char** data_ptrs, char** coding_ptrs, int size, int packetsize);
/* jerasure.cpp:1153-1176 (one super-packet at ptrs) and :1178-1192 */
ECGPU_API int ecgpu_jerasure_do_scheduled_operations(char** ptrs, int** operations, int packetsize);
ECGPU_API int ecgpu_jerasure_schedule_encode(int k, int m, int w, int** schedule, char** data_ptrs, char** coding_ptrs,
                                             int size, int packetsize);
/* A schedule over size/(w*packetsize) super-packets of nptrs devices (NULL
 * where unused): the engine behind schedule_encode and the scheduled decodes
 * (jerasure.cpp:935-995, whose schedules are built on the host). */
ECGPU_API int ecgpu_schedule_run(int nptrs, char** ptrs, int** operations, int w, int size, int packetsize);
/* Schedule construction (host) and scheduled decoding (host schedule, GPU
 * execution): jerasure.cpp:1194-1224, :1226-1344, :534-541, :997-1032,
 * :543-559 (returns ECGPU_ERR_ARG for m != 2 instead of exit), :935-961,
 * :963-995.  Schedules are the reference's malloc'd int** (rows of 5,
 * terminated by a row starting with -1). */
ECGPU_API int** ecgpu_jerasure_dumb_bitmatrix_to_schedule(int k, int m, int w, int* bitmatrix);
ECGPU_API int** ecgpu_jerasure_smart_bitmatrix_to_schedule(int k, int m, int w, int* bitmatrix);
ECGPU_API void ecgpu_jerasure_free_schedule(int** schedule);
ECGPU_API int*** ecgpu_jerasure_generate_schedule_cache(int k, int m, int w, int* bitmatrix, int smart);
ECGPU_API int ecgpu_jerasure_free_schedule_cache(int k, int m, int*** cache);
ECGPU_API int ecgpu_jerasure_schedule_decode_lazy(int k, int m, int w, int* bitmatrix, int* erasures, char** data_ptrs,
                                                  char** coding_ptrs, int size, int packetsize, int smart);
ECGPU_API int ecgpu_jerasure_schedule_decode_cache(int k, int m, int w, int*** scache, int* erasures, char** data_ptrs,
                                                   char** coding_ptrs, int size, int packetsize);
/* jerasure.cpp:1143-1151: fills xor, gf, memcpy byte counts and resets. */
ECGPU_API int ecgpu_jerasure_get_stats(double* fill_in);

/* ---------------------- hot path: batched, device-resident, async ------- */
/* A plan = one rows x nsrc GF(2^8) coefficient matrix (uploaded once) bound
 * to a table of device pointers for `stripes` stripes:
 *     dst[s][r] = XOR_j coefs[r][j] * src[s][j]   over `size` bytes.
 * Launches are asynchronous on the given hipStream_t (NULL = default stream)
 * and graph-capturable once bound.  ecgpu_plan_create enqueues the
 * coefficient-table upload on a per-device stream and returns; ecgpu_plan_bind
 * (blocking) waits for it, so a bound plan's launches never wait on the host.
 * SURVEY.md §8b "batched device API". */
typedef struct ecgpu_plan ecgpu_plan;
ECGPU_API ecgpu_plan* ecgpu_plan_create(int rows, int nsrc, const int* coefs, int device);
ECGPU_API int ecgpu_plan_bind(ecgpu_plan* p, int stripes, const uint8_t* const* src_ptrs, uint8_t* const* dst_ptrs,
                              int64_t size);
/* The buffer contract of a bind (host only; ecgpu_plan_bind and
 * ecgpu_encode_batch run it first): ECGPU_ERR_ARG, naming the pair in
 * ecgpu_last_error(), when an output shares a byte with another buffer of the
 * bind -- except an output identical to a source of its own stripe with
 * rows <= 4 (one launch; each column is read before it is written).  The
 * synchronous calls above apply the same rule (identical or disjoint):
 * identical pointers follow the reference's sequential semantics, partially
 * overlapping regions that are written are rejected, because the reference's
 * bytes for them depend on its loop order (galois.cpp:452-465, :731-754). */
ECGPU_API int ecgpu_plan_check_buffers(int rows, int nsrc, int stripes, const uint8_t* const* src_ptrs,
                                       uint8_t* const* dst_ptrs, int64_t size);
/* kind: ECGPU_KERNEL_PERM (production) or ECGPU_KERNEL_LDS; nontemporal: store
 * cache policy of the production kernel: 0 plain, 1 non-temporal (the
 * default; larger values clamp to 1); its loads are always non-temporal. */
ECGPU_API int ecgpu_plan_set_kernel(ecgpu_plan* p, int kind, int nontemporal);
ECGPU_API int ecgpu_plan_launch(ecgpu_plan* p, void* stream);
ECGPU_API void ecgpu_plan_destroy(ecgpu_plan* p);

/* ECX-style incremental parity accumulation (ecx_datanode_main.cpp:680-735)
 * with the m accumulators resident in HBM.  Source blocks arrive one at a
 * time (host or device memory); each ecgpu_accum_add is ONE fused launch
 * that updates all m accumulators with the reference's per-accumulator
 * first-touch semantics: coefficient 0 leaves an accumulator untouched, 1
 * copies (first touch) or XORs, anything else multiplies (first touch) or
 * multiply-XORs.  Only the block crosses PCIe per arrival; parity is read
 * out once with ecgpu_accum_read.  ecgpu_accum_add is synchronous;
 * ecgpu_accum_add_async only queues the block's copy and its update on the
 * accumulator's own stream and returns, so consecutive blocks cross PCIe back
 * to back with no host round trip per block -- its block must stay valid and
 * unchanged until ecgpu_accum_sync, a read, a reset or a synchronous add
 * returns (each of which waits for every queued add). */
typedef struct ecgpu_accum ecgpu_accum;
ECGPU_API ecgpu_accum* ecgpu_accum_create(int m, int64_t size, int device);
ECGPU_API int ecgpu_accum_add(ecgpu_accum* a, const char* block, const int* coefs /* m */);
ECGPU_API int ecgpu_accum_add_async(ecgpu_accum* a, const char* block, const int* coefs /* m */);
ECGPU_API int ecgpu_accum_sync(ecgpu_accum* a);
ECGPU_API int ecgpu_accum_read(ecgpu_accum* a, int i, char* out, int64_t nbytes); /* -1 if never touched */
ECGPU_API char* ecgpu_accum_device_ptr(ecgpu_accum* a, int i);
ECGPU_API int ecgpu_accum_reset(ecgpu_accum* a);
ECGPU_API void ecgpu_accum_destroy(ecgpu_accum* a);

/* Host-memory stripe pipeline (the client write path, client_main.cpp:
 * 1714-1815): stripes whose shards live in host memory are encoded with the
 * H2D copy of stripe i+1, the encode of stripe i and the D2H copy of stripe
 * i-1 overlapped on three HIP streams over a `depth`-deep ring of device
 * stripe buffers.  submit returns a ticket at once; the caller's buffers must
 * stay valid and unmodified until ecgpu_pipeline_wait(ticket) returns, after
 * which the parity is in coding_ptrs.  Copies are asynchronous DMA for pinned
 * memory (see ecgpu_host_register) and HIP-staged for pageable memory. */
typedef struct ecgpu_pipeline ecgpu_pipeline;
ECGPU_API ecgpu_pipeline* ecgpu_pipeline_create(int k, int m, const int* matrix, int64_t size, int depth,
                                                int device);
/* Read path (client_main.cpp:2055-2182, decode after recv): the same ring
 * running the fused map of jerasure_matrix_decode (jerasure.cpp:153-254) for
 * one erasure pattern.  submit takes the caller's full data_ptrs[k] /
 * coding_ptrs[m] like the reference decode: the survivors it reads are copied
 * in, the erased shards are written back in place.  NULL (ecgpu_last_error)
 * where the reference decode returns -1. */
ECGPU_API ecgpu_pipeline* ecgpu_pipeline_create_decode(int k, int m, int w, const int* matrix, int row_k_ones,
                                                       const int* erasures, int64_t size, int depth, int device);
ECGPU_API int64_t ecgpu_pipeline_submit(ecgpu_pipeline* p, char** data_ptrs, char** coding_ptrs); /* <0: error */
ECGPU_API int ecgpu_pipeline_wait(ecgpu_pipeline* p, int64_t ticket);
ECGPU_API int ecgpu_pipeline_drain(ecgpu_pipeline* p);
ECGPU_API void ecgpu_pipeline_destroy(ecgpu_pipeline* p);
/* Several GPUs from one process: stripes are independent, so
 * a group of single-device pipelines (one per entry of devices[], repeats
 * allowed) takes them round-robin -- stripe ticket t runs on member t % ndev.
 * No collective, no cross-device traffic; submit only enqueues asynchronous
 * work, so one host thread drives every device.  Same buffer rules and
 * results as ecgpu_pipeline_*; wait(t) returns once stripe t is complete. */
typedef struct ecgpu_pipeline_group ecgpu_pipeline_group;
ECGPU_API ecgpu_pipeline_group* ecgpu_pipeline_group_create(int k, int m, const int* matrix, int64_t size, int depth,
                                                            int ndev, const int* devices);
ECGPU_API ecgpu_pipeline_group* ecgpu_pipeline_group_create_decode(int k, int m, int w, const int* matrix,
                                                                   int row_k_ones, const int* erasures, int64_t size,
                                                                   int depth, int ndev, const int* devices);
ECGPU_API int64_t ecgpu_pipeline_group_submit(ecgpu_pipeline_group* g, char** data_ptrs, char** coding_ptrs);
ECGPU_API int ecgpu_pipeline_group_wait(ecgpu_pipeline_group* g, int64_t ticket);
ECGPU_API int ecgpu_pipeline_group_drain(ecgpu_pipeline_group* g);
ECGPU_API int ecgpu_pipeline_group_size(ecgpu_pipeline_group* g);
ECGPU_API void ecgpu_pipeline_group_destroy(ecgpu_pipeline_group* g);
/* The PCI bus id ("domain:bus:device.function") of a device
 * (hipDeviceGetPCIBusId): which physical GPU a rank ran on (bench.py). */
ECGPU_API int ecgpu_device_pci_bus_id(int device, char* buf, int len);
/* Page-lock caller memory for asynchronous DMA (hipHostRegister). */
ECGPU_API int ecgpu_host_register(void* ptr, int64_t bytes);
ECGPU_API int ecgpu_host_unregister(void* ptr);

/* HBM layout advice for callers that allocate their own shard slabs:
 * the byte distance to put between consecutive shards (and stripes) of
 * `size`-byte shards: round_up(size, 256) plus a skew.  Shards at
 * power-of-two strides send a column's k+m accesses to the same HBM channel /
 * bank on different rows; the skew comes from a per-size table measured on
 * MI355X (6 KiB at 4 MiB, 8 KiB at 16 MiB, none at 1 MiB; none up to 256 KiB,
 * where a stripe is one short contiguous run, and at 512 KiB; 10 KiB for
 * other sizes; shard_stride.hpp). */
ECGPU_API int64_t ecgpu_recommended_shard_stride(int64_t size);
/* The same for a known scheme: RS(k, m) slabs, where the measured best skew
 * differs by scheme (RS(10,4) keeps +12 KiB at 256 KiB and +8 KiB at 512 KiB;
 * other schemes none there).  k <= 0 = the size-only advice. */
ECGPU_API int64_t ecgpu_recommended_shard_stride_km(int64_t size, int k, int m);

/* Convenience: encode `stripes` device-resident stripes with the m x k
 * coding matrix (pointer tables are host arrays of device pointers, stripe-
 * major: data[s*k + j], coding[s*m + i]).  Asynchronous on `stream`. */
ECGPU_API int ecgpu_encode_batch(int k, int m, const int* matrix, int stripes, const uint8_t* const* data,
                                 uint8_t* const* coding, int64_t size, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ECGPU_H */
