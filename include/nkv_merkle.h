/*
 * nkv_merkle.h -- C-ABI of libnkvmerkle.so, the MI355X (gfx950) Merkle step of
 * nakevaleng's SSTable build.
 *
 * This is the drop-in boundary for the reference's ds/merkletree package
 * (magley/nakevaleng, Go).  A Go cgo shim keeps the exact Go
 * API -- NewLeaf / New / (*MerkleTree).Serialize / Deserialize / Validate --
 * and calls the entry points below; the C++ header nkv_merkletree.hpp is the
 * same shim for C++ hosts.  Paths in the citations are relative to the
 * reference root.
 *
 *   reference symbol                                   replaced by
 *   ------------------------------------------------   -------------------------------
 *   merkletree.NewLeaf      ds/merkletree/merklenode.go:27-34   nkv_leaf_hash (batched)
 *   merkletree.New / build  ds/merkletree/merkletree.go:18-64   nkv_tree_build, nkv_tree_generic
 *   NewLeaf loop + New      core/sstable/sstable.go:58-71       nkv_tree_from_values
 *   (*MerkleTree).Serialize ds/merkletree/merkletree.go:67-92   image from the calls above +
 *                           ds/merkletree/merklenode.go:37-63   nkv_write_file
 *   MakeTableSecondaries    core/sstable/sstable.go:35-47       nkv_tree_from_values /
 *     (Merkle part) + lsmtree.merge leaf collection               nkv_tree_from_records[_dev]
 *                           core/lsmtree/lsmtree.go:146,211
 *   (*MerkleTree).Validate  ds/merkletree/merkletree.go:162-171 nkv_tree_validate (device rebuild
 *                           ds/merkletree/merklenode.go:99-108    + 20-byte root compare)
 *   compaction over GPUs    core/lsmtree/lsmtree.go:71-128,211  nkv_group_* (one process, one
 *                core/sstable/sstable.go:35-47       context per GPU, RCCL)
 *   record value location   core/record/record.go:191-199       nkv_locate_values_dev
 *   bloomfilter.New sizing  ds/bloomfilter/bloomfilter.go:18-24 nkv_bloom_params
 *   makeFilter / Insert     core/sstable/sstable.go:49-56,      nkv_bloom_build /
 *                           ds/bloomfilter/bloomfilter.go:76-91 nkv_bloom_from_records /
 *                                                               nkv_bloom_insert[_records]_dev
 *   (*BloomFilter).Query    ds/bloomfilter/bloomfilter.go:93-111 nkv_bloom_query_dev
 *   record checksum         core/record/record.go:51 (New),     nkv_record_crc /
 *     crc32.ChecksumIEEE    :163-169 (Deserialize check)        nkv_record_crc_dev /
 *     over Key ++ Value                                         nkv_crc32_dev
 *
 * Conventions
 *   - Every function returns an nkv_status (0 = NKV_OK) unless noted; nothing
 *     aborts.  nkv_strerror() gives the message; NKV_ERR_EMPTY's message is
 *     the reference's exact error text (merkletree.go:20).
 *   - Digests are 20 bytes in Go's byte order (sha1.Sum output).
 *   - "nodes" buffers hold every tree level bottom-up, level-major: level L
 *     has nkv_level_count(n, L) digests starting at digest index
 *     nkv_level_start(n, L); level 0 is the leaves, the root is the last
 *     digest (index nkv_total_nodes(n) - 1).  Pads are not stored.
 *   - "img" buffers receive the exact byte image Serialize() writes
 *     (nkv_bfs_size(n) bytes for 20-byte leaves).
 *   - Host-pointer functions are synchronous: outputs are written before
 *     return, and no caller pointer is retained (cgo rule).  Inputs are
 *     staged through library-owned pinned memory: a pool of host threads
 *     gathers chunk k+1 while chunk k is copied to the device.
 *   - *_dev functions take device pointers and are asynchronous on the
 *     context's stream (nkv_ctx_set_stream); nkv_ctx_sync() waits.
 *   - Thread safety: distinct contexts may be used concurrently; one context
 *     must not be used by two threads at once.  Every call re-binds the
 *     context's device (cgo calls may land on any OS thread).
 */
#ifndef NKV_MERKLE_H
#define NKV_MERKLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NKV_DIGEST_SIZE 20
#define NKV_MERKLE_NODE_EMPTY 1 /* merklenode.go:11 */

typedef enum nkv_status {
    NKV_OK = 0,
    NKV_ERR_EMPTY = 1,   /* "cannot build Merkle Tree from 0 nodes" (merkletree.go:20) */
    NKV_ERR_INVALID = 2, /* bad argument (null pointer, size overflow, bad record,
                            more than 2^31 - 1 values in one batch) */
    NKV_ERR_DEVICE = 3,  /* HIP runtime / kernel launch failure, or no such device */
    NKV_ERR_NOMEM = 4,   /* device, pinned-host or host allocation failed */
    NKV_ERR_IO = 5       /* file open/write failed (nkv_write_file) */
} nkv_status;

typedef struct nkv_ctx nkv_ctx;

/* ---- ABI version ----
 * NKV_ABI_VERSION is the version this header describes; nkv_abi_version()
 * the one the loaded library implements.  A caller built against version V
 * checks nkv_abi_version() == V at start (the Go shim does).
 * The version goes up whenever an existing entry point changes its meaning or
 * signature; adding entry points or option values does not change it.
 *   1: nkv_group_tree_dev takes d_roots as an array of g device pointers
 *      (void *const *; before: one device pointer), and the options
 *      NKV_OPT_DEEP_PREFETCH / NKV_OPT_QUEUE_RING accept only their one
 *      remaining value (and, since round 6, NKV_OPT_QUEUE_PAIR only 0: the
 *      opt-in pair kernel it selected never passed a GPU run). */
#define NKV_ABI_VERSION 1
int nkv_abi_version(void);

/* ---- errors, devices, contexts ---- */
const char *nkv_strerror(int status);
/* "nkv-src-sha256:<64 hex>": SHA-256 of the sources and build flags this
 * library was compiled from (nakevaleng_amd/build.py checks it before use). */
const char *nkv_build_id(void);
int nkv_device_count(int *count);
int nkv_ctx_create(int device, nkv_ctx **out);
void nkv_ctx_destroy(nkv_ctx *ctx);
/* Work is issued on the context's own (non-blocking) stream until
 * nkv_ctx_set_stream() selects a hipStream_t of the context's device; NULL
 * selects the device's null stream.  nkv_ctx_use_own_stream() switches back. */
int nkv_ctx_set_stream(nkv_ctx *ctx, void *hip_stream);
int nkv_ctx_use_own_stream(nkv_ctx *ctx);
int nkv_ctx_sync(nkv_ctx *ctx);
/* Tuning knobs (defaults are the measured-best settings). */
#define NKV_OPT_LEAF_LOAD 1 /* leaf-kernel load path: 4 (default) = 16-byte aligned values in
                               128-byte runs straight into registers, others as 11; 11 =
                               every value through the staged paths: the segment stage
                               when a wave's values share their offset mod 64, the
                               80-byte window stage when their full-block counts are
                               equal, else the value-relative LDS-DMA stream.  (The
                               load paths that lost their A/Bs in rounds 1-2 are gone.) */
#define NKV_OPT_BUCKET 2    /* ragged values (nkv_tree_from_values*, nkv_tree_from_records*):
                               1 = hash in length-sorted order (work queue); 0 = in input
                               order; 2 (default) = auto: input order when the full-block
                               counts of a batch of >= 4096 values lie within max(1, min/16)
                               of each other, else sorted (decided on the device, no
                               read-back) */
#define NKV_OPT_DEEP_PREFETCH 3 /* retired (ABI version 1): 3 is the only value accepted */
#define NKV_OPT_QUEUE_RING 9    /* retired (ABI version 1): 13 is the only value accepted */
#define NKV_OPT_QUEUE_SPLIT 4 /* work-queue kernel: groups whose longest value has at most
                                 this many 64-B blocks may go to the non-priority waves
                                 when the longest value bounds the batch (default 32) */
#define NKV_OPT_QUEUE_WAVES 5 /* work-queue kernel: waves per SIMD, 1..3 (default 3: its
                                 3-slot, 12 KiB LDS ring per wave) */
#define NKV_OPT_CRC_LOAD 6    /* record checksums: 0 (default) = one lane per span, slicing-by-4
                                 from lane-private LDS table columns (no bank conflicts),
                                 whole 128-byte lines into registers; 8 = 16 lanes per span,
                                 chunk states combined by CRC advance tables (a few long
                                 spans) */
#define NKV_OPT_HOST_THREADS 7 /* host-buffer API: threads that gather caller bytes into the
                                  pinned staging chunks (0 = default: min(16, cores), or
                                  the NKV_HOST_THREADS environment variable) */
#define NKV_OPT_STAGE_CHUNK 8  /* host-buffer API: bytes per pinned staging chunk (multiple of
                                  4096, default 32 MiB; three chunks are in flight) */
#define NKV_OPT_BLOOM_PATH 10  /* filter inserts: 2 (default) = group the bit updates by 32768-bit
                                  range from one hash pass (each tile counting-sorted in LDS and
                                  staged), then set them in LDS, one workgroup per range; 1 = the
                                  same grouping by a global counting sort (hashes twice); 0 = one
                                  device atomicOr per bit */
#define NKV_OPT_RECORDS_FUSED 11 /* records form (nkv_tree_from_records*): 1 (default) = one
                                    launch locates each value from its header and hashes it
                                    (k_leaf_records); 0 = a separate locate pass first */
#define NKV_OPT_TABLE_LANES 12 /* nkv_trees_dev: streams the tables of one call are spread
                                  over (1..8, default 2), so one table's leaf kernel runs
                                  while the previous one finishes and reduces */
#define NKV_OPT_TIMING_EVERY 13 /* NKV_TIMING_EVENTS on every k-th tree call only (1..10^6,
                                   default 1; counted from nkv_ctx_set_timing): each event
                                   record is a packet on the stream between two kernels,
                                   so a timed loop samples its kernel times instead of
                                   carrying three records per call */
#define NKV_OPT_SMALL_PATH 14 /* host-buffer tree calls (nkv_tree_from_values, nkv_tree_from_records)
                                 of at most NKV_OPT_SMALL_MAX_N values and NKV_OPT_SMALL_MAX_BYTES
                                 of payload: the whole tree and its image in ONE launch, one
                                 synchronize.  1 (default) = the kernel reads the packed values
                                 and writes its results across PCIe (host-coherent pinned
                                 buffers, no DMA); 2 = one copy to HBM, the launch, one copy
                                 back; 3 = the resident service: one workgroup stays on the GPU
                                 and serves each call of at most 256 values from a mailbox
                                 (NKV_OPT_SERVICE_MAILBOX) as path 1 does, without a launch or the runtime's
                                 completion (larger calls take path 1; the service leaves
                                 20 ms after its last request, or at nkv_ctx_destroy, and the
                                 next call starts it again; while it runs, a device-wide
                                 synchronize waits for it to leave); 0 = off (the grid path
                                 for every size) */
#define NKV_OPT_SMALL_MAX_N 15     /* 0..1024 (default 1024) */
#define NKV_OPT_SMALL_MAX_BYTES 16 /* payload bound of the small path (default 1 MiB; the values
                                      16-byte aligned; for records the whole stream) */
#define NKV_OPT_ARENA_COHERENT 17   /* nkv_host_alloc blocks: 1 (default) = host-coherent pinned memory
                                       (copies read it as any pinned block, and the small path's kernel
                                       reads NewLeaf values in place); 0 = default pinned memory */
#define NKV_OPT_SIDE_GATE 18 /* device-length batches on the gated plan (NKV_OPT_BUCKET 2): 1 (default) =
                                the input-order leaf kernel runs on a second stream of the context,
                                beside the length sort and the work queue (whichever of the two the
                                device-side range opens does the work; the other exits), joined
                                before the levels; 0 = all of them in turn on the context's stream */
#define NKV_OPT_QUEUE_PAIR 19 /* retired (ABI version 1): 0 is the only value accepted (one wave per
                                 work-queue group; the two-wave pair kernel of round 5 was removed
                                 after failing its first GPU parity run) */
#define NKV_OPT_SERVICE_MAILBOX 20 /* where small-tree calls put their input: 0 (default) = in
                                      fine-grained device memory the host stores to directly,
                                      when the GPU has a large BAR and the packed input fits
                                      16 KiB (the kernel stages local memory instead of reading
                                      across PCIe; for the resident service, NKV_OPT_SMALL_PATH 3,
                                      its doorbell and request line too, so it polls local
                                      memory; else as 1); 1 = in host-coherent memory.  Answers
                                      always land in host memory.  A change stops a running
                                      service; the next call starts it in the new form */
int nkv_ctx_set_option(nkv_ctx *ctx, int key, int64_t value);
/* Which path the latest host-buffer tree call of the context took */
#define NKV_PATH_GRID 0  /* copies + leaf kernel + per-level reduce launches */
#define NKV_PATH_SMALL 1 /* the one-launch small tree (NKV_OPT_SMALL_PATH) */
int nkv_ctx_last_path(nkv_ctx *ctx, int *path);
/* The resident small-tree service of the context (NKV_OPT_SMALL_PATH 3), for
 * diagnostics: out[0] doorbell (latest request), out[1] served (the latest the
 * service took), out[2] done (the latest it answered), out[3] launches so far,
 * out[4] 1 while a launch may still run, out[5] 1 if its stream still has work,
 * out[6] 1 if its requests go through device memory (NKV_OPT_SERVICE_MAILBOX),
 * out[7] where its latest launch landed: XCC_ID << 32 | HW_ID (the hardware's
 * wave/SIMD/CU/SE word).  All zero before the first request. */
int nkv_ctx_small_service_state(nkv_ctx *ctx, uint64_t out[8]);
/* Diagnostics of the same service: enable = 1 makes it stamp the phases of
 * each following request; out (nullable) receives the latest traced request's
 * stamps, seven (s_memrealtime at 100 MHz, s_memtime in shader clocks) pairs:
 * doorbell seen, input staged, leaves hashed, levels + image written,
 * completion stored, then levels done and first image segment built. */
int nkv_ctx_small_service_trace(nkv_ctx *ctx, int enable, uint64_t out[14]);
/* Timing (nkv_ctx_set_timing flags).  NKV_TIMING_EVENTS: the tree calls record
 * HIP events around the leaf kernel and the tree reduce on the context's
 * stream (and, for nkv_tree_from_values, around the upload and the download).
 * NKV_TIMING_CLOCK: every wave of the leaf kernels on the context's device
 * adds its lifetime in shader-clock cycles and in 100 MHz ticks to a
 * counter the context owns (nkv_ctx_clock); one context per device at a
 * time.  0 switches both off. */
#define NKV_TIMING_EVENTS 1
#define NKV_TIMING_CLOCK 2
int nkv_ctx_set_timing(nkv_ctx *ctx, int flags);
/* the latest tree call that recorded events (every call, or every k-th under
 * NKV_OPT_TIMING_EVERY) */
int nkv_ctx_last_timing(nkv_ctx *ctx, float *leaf_ms, float *reduce_ms);
/* the latest nkv_tree_from_values under NKV_TIMING_EVENTS: upload (host values ->
 * HBM), kernels (leaf + tree), download (outputs -> host); NKV_ERR_INVALID when
 * that call was not sampled (NKV_OPT_TIMING_EVERY) */
int nkv_ctx_last_host_timing(nkv_ctx *ctx, float *upload_ms, float *kernels_ms, float *download_ms);
/* NKV_TIMING_CLOCK: the lifetime-weighted mean shader clock of the leaf-kernel
 * waves since the flag was set, and how many waves reported (synchronizes). */
int nkv_ctx_clock(nkv_ctx *ctx, double *mhz, uint64_t *waves);
/* Sum over every tree call since timing was (re-)enabled: synchronizes on the
 * last call's events only, so a timed loop is not perturbed. */
int nkv_ctx_timing_summary(nkv_ctx *ctx, int *calls, float *leaf_ms_total, float *reduce_ms_total);

/* ---- tree shape (pure, no device) ---- */
int nkv_num_levels(uint64_t n); /* incl. the leaf level; 0 for n == 0 */
uint64_t nkv_level_count(uint64_t n, int level);
uint64_t nkv_level_start(uint64_t n, int level);
uint64_t nkv_total_nodes(uint64_t n);
uint64_t nkv_bfs_size(uint64_t n); /* Serialize() bytes for 20-byte leaves */

/* ---- pinned host arena (for the deferred-NewLeaf shim) ----
 * A block from nkv_host_alloc belongs to the context.  Host-buffer calls on the
 * same context whose values all lie inside one block copy them to the device
 * in one DMA straight from the block (no staging gather), values keeping their
 * places (16-byte aligned places take the aligned kernel path).
 * nkv_host_stream(block, upto): bytes [0, upto) of the block are final for the
 * current batch; their copy to the device starts now, asynchronously, so it
 * overlaps the caller's NewLeaf loop; the next call over the block moves only
 * the rest.  Those bytes must not change until that call returns.  A call over
 * the block ends the batch; an upto below the previous one starts a new batch.
 * nkv_host_free waits for copies from the block.  For a block of at least
 * 64 MiB nkv_host_alloc also allocates its device mirror (as many bytes of
 * HBM), so a block reserved once (e.g. at engine start, from the memtable's
 * capacity) costs the flushes that use it no allocation; smaller blocks, or a
 * mirror that does not fit the free HBM at that moment, get it on first use
 * (values that take the small path never need it). */
int nkv_host_alloc(nkv_ctx *ctx, uint64_t bytes, void **out);
int nkv_host_free(nkv_ctx *ctx, void *p);
int nkv_host_stream(nkv_ctx *ctx, const void *block, uint64_t upto);

/* ---- host-buffer API (synchronous) ---- */

/* NewLeaf over n values: value i = base[off[i] .. off[i]+len[i]).
 * out20: n * 20 bytes. */
int nkv_leaf_hash(nkv_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint64_t *len,
                  uint64_t n, uint8_t *out20);

/* New() over n NewLeaf digests (leaf20: n * 20 bytes).  Outputs are
 * optional (NULL to skip): root20 (20 B), nodes_out (nkv_total_nodes(n) * 20 B),
 * img_out (nkv_bfs_size(n) B). */
int nkv_tree_build(nkv_ctx *ctx, const uint8_t *leaf20, uint64_t n, uint8_t *root20,
                   uint8_t *nodes_out, uint8_t *img_out);

/* makeMetadata: NewLeaf(value_i) for all i, then New, then the Serialize
 * image -- in one call. */
int nkv_tree_from_values(nkv_ctx *ctx, const uint8_t *base, const uint64_t *off,
                         const uint64_t *len, uint64_t n, uint8_t *root20, uint8_t *nodes_out,
                         uint8_t *img_out);

/* New() over leaves with arbitrary Data (leaf i = data[off[i] .. +len[i]),
 * README example ds/merkletree/README.md:44-57).  upper_out receives levels
 * 1..top ((nkv_total_nodes(n) - n) * 20 B).  img_out receives the Serialize
 * image (length nkv_generic_bfs_size()). */
uint64_t nkv_generic_bfs_size(const uint64_t *len, uint64_t n);
int nkv_tree_generic(nkv_ctx *ctx, const uint8_t *data, const uint64_t *off, const uint64_t *len,
                     uint64_t n, uint8_t *root20, uint8_t *upper_out, uint8_t *img_out);

/* (*MerkleTree).Validate (merkletree.go:162-171) of a tree New built from n
 * leaves: rehash (merklenode.go:99-108) recomputes every internal node from
 * the leaves' Data -- leaf i = leaf_data[off[i] .. off[i]+len[i]), a NewLeaf
 * leaf is its 20-byte digest, any other length is a generic leaf (README
 * example); pads contribute no bytes -- on the device, and compares the 20
 * bytes with root20 (the tree's Root.Data).  *ok = 1 if they match, else 0. */
int nkv_tree_validate(nkv_ctx *ctx, const uint8_t *leaf_data, const uint64_t *off, const uint64_t *len,
                      uint64_t n, const uint8_t *root20, int *ok);

/* Merkle step straight from a serialized Data-table stream (the records
 * written by record.Serialize, record.go:191-199) and the RecSize of each
 * record (record.KeyContext, record.go:38-41).  Leaves are the record Values
 * (sstable.go:62, lsmtree.go:211), hashed in place on the device. */
int nkv_tree_from_records(nkv_ctx *ctx, const uint8_t *stream, uint64_t stream_len,
                          const uint64_t *rec_size, uint64_t n, uint8_t *root20,
                          uint8_t *nodes_out, uint8_t *img_out);

/* Record checksums: CRC-32/IEEE of Key ++ Value of each
 * serialized record (stream and rec_size as for nkv_tree_from_records).
 * crc_out (nullable): n checksums, what record.New stores (record.go:51).
 * *n_bad: records whose stored Crc differs from the recomputed one, the check
 * record.Deserialize panics on (record.go:163-169); *first_bad: the lowest such
 * index, UINT64_MAX if none.  NKV_ERR_INVALID if a header points outside the
 * stream. */
int nkv_record_crc(nkv_ctx *ctx, const uint8_t *stream, uint64_t stream_len,
                   const uint64_t *rec_size, uint64_t n, uint32_t *crc_out, uint64_t *n_bad,
                   uint64_t *first_bad);

/* SSTable filter.  bloomfilter.New(n, p)'s sizing: m bits,
 * k hash functions (bloomfilter.go:18-24; n > 0, 0 < p < 1).  Hash j of a key is
 * MurmurHash3_x86_32(key, seed0 + j) % m (spaolacci/murmur3 Sum32; the reference
 * draws seed0 = uint32(time.Now().UnixNano()), bloomfilter.go:31 -- here it is
 * an argument).  Bit idx is Contents[idx / 8] & (1 << (idx % 8)). */
int nkv_bloom_params(uint64_t n, double p, uint32_t *m, uint32_t *k);
/* makeFilter over n keys (key i = keys + off[i], len[i]): bits_out receives
 * Contents, ceil(m / 8) bytes (bloomfilter.go:67). */
int nkv_bloom_build(nkv_ctx *ctx, const uint8_t *keys, const uint64_t *off, const uint64_t *len,
                    uint64_t n, uint32_t m, uint32_t k, uint32_t seed0, uint8_t *bits_out);
/* makeFilter over the keys of serialized records (stream and rec_size as for
 * nkv_tree_from_records; sstable.go:51-53 inserts KeyContext.Key). */
int nkv_bloom_from_records(nkv_ctx *ctx, const uint8_t *stream, uint64_t stream_len,
                           const uint64_t *rec_size, uint64_t n, uint32_t m, uint32_t k,
                           uint32_t seed0, uint8_t *bits_out);

/* Serialize()'s file semantics: open O_WRONLY|O_CREAT (mode 0666) WITHOUT
 * O_TRUNC (merkletree.go:68), write len bytes at offset 0, close. */
int nkv_write_file(const char *fname, const uint8_t *data, uint64_t len);

/* ---- device-resident API (asynchronous on the context stream) ---- */

/* level 0 of d_nodes from n values at d_base + d_off[i], d_len[i] (any alignment) */
int nkv_leaf_hash_dev(nkv_ctx *ctx, const void *d_base, const uint64_t *d_off,
                      const uint64_t *d_len, uint64_t n, void *d_nodes);
/* level 0 of d_nodes from n values of len bytes at d_base + i * stride */
int nkv_leaf_hash_strided_dev(nkv_ctx *ctx, const void *d_base, uint64_t stride, uint64_t len,
                              uint64_t n, void *d_nodes);
/* levels 1..top of d_nodes from its level 0 */
int nkv_tree_reduce_dev(nkv_ctx *ctx, void *d_nodes, uint64_t n);
/* leaf hash (order per NKV_OPT_BUCKET), then the tree levels */
int nkv_tree_from_values_dev(nkv_ctx *ctx, const void *d_base, const uint64_t *d_off,
                             const uint64_t *d_len, uint64_t n, void *d_nodes);
int nkv_tree_from_strided_dev(nkv_ctx *ctx, const void *d_base, uint64_t stride, uint64_t len,
                              uint64_t n, void *d_nodes);
/* Serialize() image of a 20-byte-leaf tree (nkv_bfs_size(n) bytes) */
int nkv_bfs_image_dev(nkv_ctx *ctx, const void *d_nodes, uint64_t n, void *d_img);
/* d_rec_off[i] = sum of d_rec_size[0..i) (exclusive scan of KeyContext.RecSize) */
int nkv_record_offsets_dev(nkv_ctx *ctx, const uint64_t *d_rec_size, uint64_t n,
                           uint64_t *d_rec_off);
/* value offset/length of each record; NKV_ERR_INVALID (after a sync) if a
 * header points outside the stream */
int nkv_locate_values_dev(nkv_ctx *ctx, const void *d_stream, uint64_t stream_len,
                          const uint64_t *d_rec_off, uint64_t n, uint64_t *d_voff,
                          uint64_t *d_vlen);
/* Merkle step of a device-resident Data table (compaction, lsmtree.go:211 /
 * sstable.go:41-46), asynchronous: the Value of each record at d_stream +
 * d_rec_off[i] (record.go:191-199) is located and hashed in place, and the full
 * tree goes to d_nodes.  d_err (nullable, 4 bytes on the device) receives 1 if
 * a header points outside the stream (that leaf hashes the empty value); with
 * d_err NULL the call synchronizes and returns NKV_ERR_INVALID instead. */
int nkv_tree_from_records_dev(nkv_ctx *ctx, const void *d_stream, uint64_t stream_len,
                              const uint64_t *d_rec_off, uint64_t n, void *d_nodes, uint32_t *d_err);
/* CRC-32/IEEE (Go crc32.ChecksumIEEE) of n byte spans d_base + d_off[i],
 * d_len[i] (any alignment) into d_crc[i] */
int nkv_crc32_dev(nkv_ctx *ctx, const void *d_base, const uint64_t *d_off, const uint64_t *d_len,
                  uint64_t n, uint32_t *d_crc);
/* Record checksums over Key ++ Value of the records at d_stream + d_rec_off[i].
 * d_crc (nullable): n checksums.  d_stats (nullable, 3 x u64 on the device,
 * overwritten): [0] records whose stored Crc differs, [1] the lowest such index
 * (UINT64_MAX if none), [2] 1 if a header points outside the stream. */
int nkv_record_crc_dev(nkv_ctx *ctx, const void *d_stream, uint64_t stream_len,
                       const uint64_t *d_rec_off, uint64_t n, uint32_t *d_crc, uint64_t *d_stats);
/* Compaction read of a device-resident Data table in one call, asynchronous:
 * the Merkle tree of the records' Values into d_nodes (as
 * nkv_tree_from_records_dev) and record.Deserialize's checksum check
 * (record.go:163-169) of every record, d_crc / d_stats as nkv_record_crc_dev
 * (a header outside the stream sets d_stats[2]; that leaf hashes the empty
 * value).  Records of similar sizes are read once for both (k_leaf_verify). */
int nkv_tree_verify_records_dev(nkv_ctx *ctx, const void *d_stream, uint64_t stream_len,
                                const uint64_t *d_rec_off, uint64_t n, void *d_nodes, uint32_t *d_crc,
                                uint64_t *d_stats);
/* Bloom filter bits on the device: d_bits holds ((m + 31) / 32) * 4 bytes
 * (Contents padded to whole 32-bit words, zero the padding); bits are OR-ed in,
 * so several calls build one filter. */
int nkv_bloom_insert_dev(nkv_ctx *ctx, const void *d_keys, const uint64_t *d_off,
                         const uint64_t *d_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0,
                         void *d_bits);
/* keys of the records at d_stream + d_rec_off[i]; NKV_ERR_INVALID (after a
 * sync) if a header points outside the stream */
int nkv_bloom_insert_records_dev(nkv_ctx *ctx, const void *d_stream, uint64_t stream_len,
                                 const uint64_t *d_rec_off, uint64_t n, uint32_t m, uint32_t k,
                                 uint32_t seed0, void *d_bits);
/* d_out[i] = 1 if key i may be in the filter (every bit set), else 0 */
int nkv_bloom_query_dev(nkv_ctx *ctx, const void *d_keys, const uint64_t *d_off,
                        const uint64_t *d_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0,
                        const void *d_bits, uint8_t *d_out);
/* synthetic input: byte j = byte (j % 8) of splitmix64(seed, j / 8) */
int nkv_fill_splitmix64_dev(nkv_ctx *ctx, void *d_buf, uint64_t nbytes, uint64_t seed);

/* ---- several tables per call (compaction's runs, consecutive flushes) ----
 * One table of device-resident leaves, described for nkv_trees_dev /
 * nkv_group_trees_dev (all pointers on the device that builds it). */
typedef enum nkv_table_kind {
    NKV_TABLE_STRIDED = 0, /* value i = base + i * stride, len bytes (nkv_tree_from_strided_dev) */
    NKV_TABLE_VALUES = 1,  /* value i = base + off[i], lens[i] bytes (nkv_tree_from_values_dev) */
    NKV_TABLE_RECORDS = 2, /* Data table: base = stream of base_len bytes, off = record offsets
                              (nkv_tree_from_records_dev; err nullable) */
    NKV_TABLE_VERIFY = 3   /* as RECORDS plus every record's Crc checked
                              (nkv_tree_verify_records_dev; crc, stats nullable) */
} nkv_table_kind;
typedef struct nkv_table {
    int kind;
    const void *base;
    uint64_t base_len;
    uint64_t stride, len;
    const uint64_t *off;
    const uint64_t *lens;
    uint64_t n;
    void *nodes; /* nkv_total_nodes(n) * 20 bytes */
    uint32_t *err;
    uint32_t *crc;
    uint64_t *stats;
} nkv_table;
/* The trees of k independent tables, asynchronous on the context's stream:
 * the tables are spread over NKV_OPT_TABLE_LANES streams of the context's
 * device (table t on lane t % lanes, forked from and joined back to the
 * context's stream), so one table's leaf kernel overlaps the tail and the tree
 * reduce of the one before.  Each table's results are those of its single-table
 * call.  A RECORDS table with err NULL: the call synchronizes and returns
 * NKV_ERR_INVALID if any of those tables has a header outside its stream. */
int nkv_trees_dev(nkv_ctx *ctx, const nkv_table *tables, int k);

/* ---- multi-GPU: one host process, one context per GPU ----
 * A group is one context per listed device and one RCCL communicator over
 * them (ncclCommInitAll).  Tables shard with no data-path exchange; the only
 * collective is the all-gather of 20-byte roots (an RCCL group call over the
 * members' streams).  Listing a device twice is allowed (several streams on
 * one GPU, e.g. to rehearse the split on one card): RCCL cannot join one
 * device twice, so such a group gathers by device-to-device copies instead
 * (nkv_group_transport). */
typedef struct nkv_group nkv_group;
#define NKV_TRANSPORT_RCCL 1
#define NKV_TRANSPORT_COPY 2
int nkv_group_create(const int *devices, int g, nkv_group **out);
void nkv_group_destroy(nkv_group *grp);
int nkv_group_size(const nkv_group *grp);
int nkv_group_transport(const nkv_group *grp);
/* Peer access between member i's GPU and member j's: nkv_group_create enables
 * xGMI peer mappings for every pair of distinct GPUs that supports them
 * (hipDeviceEnablePeerAccess; a pair already enabled counts), so GPU-to-GPU
 * copies (nkv_group_tree_fetch, the copy transport) go over xGMI.  *state:
 * NKV_PEER_ENABLED, NKV_PEER_SAME (both members on one GPU), or NKV_PEER_NONE
 * (not mappable: copies take the runtime's staged path). */
#define NKV_PEER_NONE 0
#define NKV_PEER_ENABLED 1
#define NKV_PEER_SAME 2
int nkv_group_peer_access(const nkv_group *grp, int i, int j, int *state);
/* member i's context (owned by the group): options, streams, *_dev calls */
int nkv_group_ctx(nkv_group *grp, int i, nkv_ctx **out);
int nkv_group_sync(nkv_group *grp);
/* d_roots[i]: 20 bytes on member i.  All-gather them: d_out[i] (nullable
 * array, or entries) receives the g * 20 bytes on member i (a d_roots or d_out
 * entry that is not device memory of member i's GPU: NKV_ERR_INVALID); roots_out
 * (nullable host buffer, g * 20 bytes) a copy (then the call synchronizes,
 * else it is asynchronous on the members' streams). */
int nkv_group_roots_allgather(nkv_group *grp, const void *const *d_roots, void *const *d_out,
                              uint8_t *roots_out);
/* Compaction over GPUs (lsmtree.go:71-128 merges runs; one output table per
 * GPU): table t is built on member t % g (its pointers live on that device,
 * nkv_trees_dev there), then every table's root is all-gathered so every member
 * holds all k roots in table order.  roots_out (host, k * 20 bytes, nullable):
 * then the call synchronizes; else asynchronous on the members' streams. */
int nkv_group_trees_dev(nkv_group *grp, const nkv_table *tables, int k, uint8_t *roots_out);
/* The same from host memory (cgo: what MakeTableSecondaries holds after a
 * merge): table t = values base[t] + off[t][i], len[t][i], on member t % g, one
 * host thread per member; outputs as nkv_tree_from_values (each nullable). */
typedef struct nkv_values {
    const uint8_t *base;
    const uint64_t *off;
    const uint64_t *len;
    uint64_t n;
    uint8_t *root20;
    uint8_t *nodes_out;
    uint8_t *img_out;
} nkv_values;
int nkv_group_trees_from_values(nkv_group *grp, const nkv_values *tables, int k);
/* One table over the group (a single compaction's output table, lsmtree.go:106-110):
 * padding only happens at a level's end (merkletree.go:32-34), so the tree splits
 * at 2^k-aligned leaf ranges: member r builds levels 0..k of leaves
 * [r * span, min(n, (r + 1) * span)), span = nkv_split_span(n, g) = 2^k, k =
 * max(1, ceil(log2(ceil(n / g)))); a partial last range re-hashes its lone top node
 * up to level k; the level-k nodes are all-gathered and every member reduces the
 * top ceil(log2 G) levels (G = ceil(n / span) ranges), so every member holds the
 * root.  Outputs as nkv_tree_from_values (each nullable; all host). */
uint64_t nkv_split_span(uint64_t n, int g);
int nkv_group_tree_from_values(nkv_group *grp, const uint8_t *base, const uint64_t *off, const uint64_t *len,
                               uint64_t n, uint8_t *root20, uint8_t *nodes_out, uint8_t *img_out);
/* The same over device-resident ranges: parts[r] describes member r's leaf range
 * (a STRIDED or VALUES table whose pointers live on member r's device, n = its
 * range's length, 0 for members past the last range; nodes ignored: the group
 * keeps the levels).  d_roots (nullable array of g entries, each nullable):
 * d_roots[r] is 20 bytes on member r's device that receive the root member r
 * reduced (every member's equals the root); root20 (host, nullable): then the
 * call synchronizes, else it is asynchronous on the members' streams.
 * nkv_group_tree_fetch then copies the latest such tree's nodes (level-major,
 * nkv_total_nodes(n) * 20 bytes) and/or its Serialize image to the host; after a
 * refused or failed split call there is no latest tree and it returns
 * NKV_ERR_INVALID. */
int nkv_group_tree_dev(nkv_group *grp, const nkv_table *parts, uint64_t n, void *const *d_roots,
                       uint8_t *root20);
int nkv_group_tree_fetch(nkv_group *grp, uint8_t *nodes_out, uint8_t *img_out);

#ifdef __cplusplus
}
#endif

#endif /* NKV_MERKLE_H */
