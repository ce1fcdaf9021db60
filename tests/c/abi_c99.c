/*
 * abi_c99.c -- the C-ABI as cgo sees it.
 *
 * cgo compiles a package's preamble as C, so include/nkv_merkle.h must be
 * plain C: this file is built with gcc -std=c99 -pedantic -Werror
 * (tests/test_abi_c.py) and calls the entry points a Go shim calls for the
 * flush's Merkle step (core/sstable/sstable.go:58-74 -> nkv_tree_from_values,
 * INTEGRATION.md section 2).  Input: n values, value i of (i * 37) % 301 bytes,
 * byte j of the stream = (j * 131 + 7) & 255, packed back to back.  Output, one
 * "key value" line each: abi (nkv_abi_version), levels, total, bfs (pure shape
 * functions, no device), then -- on a GPU -- root, img_sha (a FNV-1a 64 of the
 * image, the test recomputes it from the oracle's image) and path.  Without a
 * device: "device none" and exit 0 (nkv_ctx_create must fail cleanly).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "nkv_merkle.h"

static uint64_t fnv1a64(const uint8_t *p, uint64_t n) {
    uint64_t h = 14695981039346656037ULL;
    uint64_t i;
    for (i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 1099511628211ULL;
    }
    return h;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)strtoull(argv[1], NULL, 10) : 1000;
    uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    uint64_t *len = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    uint64_t total = 0, i;
    uint8_t *base, *nodes, *img;
    uint8_t root[NKV_DIGEST_SIZE];
    nkv_ctx *ctx = NULL;
    int rc, path = -1;
    if (!off || !len) return 2;
    for (i = 0; i < n; ++i) {
        off[i] = total;
        len[i] = (i * 37) % 301;
        total += len[i];
    }
    base = (uint8_t *)malloc((size_t)total + 1);
    if (!base) return 2;
    for (i = 0; i < total; ++i) base[i] = (uint8_t)((i * 131 + 7) & 255);
    printf("abi %d\n", nkv_abi_version());
    printf("levels %d\n", nkv_num_levels(n));
    printf("total %llu\n", (unsigned long long)nkv_total_nodes(n));
    printf("bfs %llu\n", (unsigned long long)nkv_bfs_size(n));
    if (nkv_abi_version() != NKV_ABI_VERSION) return 3;
    rc = nkv_ctx_create(0, &ctx);
    if (rc != NKV_OK) {
        printf("device none (%s)\n", nkv_strerror(rc));
        return rc == NKV_ERR_DEVICE ? 0 : 4;
    }
    nodes = (uint8_t *)malloc((size_t)(NKV_DIGEST_SIZE * nkv_total_nodes(n)));
    img = (uint8_t *)malloc((size_t)nkv_bfs_size(n));
    if (!nodes || !img) return 2;
    rc = nkv_tree_from_values(ctx, base, off, len, n, root, nodes, img);
    if (rc != NKV_OK) {
        fprintf(stderr, "nkv_tree_from_values: %s\n", nkv_strerror(rc));
        return 5;
    }
    if (nkv_ctx_last_path(ctx, &path) != NKV_OK) return 6;
    printf("root ");
    for (i = 0; i < NKV_DIGEST_SIZE; ++i) printf("%02x", root[i]);
    printf("\nimg_fnv %016llx\n", (unsigned long long)fnv1a64(img, nkv_bfs_size(n)));
    printf("path %d\n", path);
    /* the empty batch: the reference's exact error (merkletree.go:20) */
    rc = nkv_tree_from_values(ctx, base, off, len, 0, root, NULL, NULL);
    printf("empty %d %s\n", rc, nkv_strerror(rc));
    nkv_ctx_destroy(ctx);
    free(nodes);
    free(img);
    free(base);
    free(off);
    free(len);
    return 0;
}
