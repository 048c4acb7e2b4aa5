/*
 * worker_harness.c -- a plain-C host that drives libmrgpu.so exactly the way the reference's Worker
 * would through an FFI crate (test of SURVEY.md §8 row f4; INTEGRATION.md shows the Rust form):
 *
 *   Worker::map(m)    src/mr/worker.rs:142-155
 *     read_file_to_mem_map        data/gut-{m}.txt, whole file            worker.rs:65-77
 *     call_map_func(wc::map) + cal_hash_for_key + write_key_value_to_file  -> mrg_map
 *   Worker::reduce(r) src/mr/worker.rs:157-193
 *     read_file_to_mem_reduce + sort + group + call_reduce_func(wc::reduce) -> mrg_reduce
 *     File::create("mr-{r}.txt") + write_all                               worker.rs:167-179
 *
 * usage: worker_harness <map_n> <reduce_n> [--indexer]   (run in a directory holding data/)
 * Map tasks run in order, then reduce tasks (the coordinator's phase barrier, coordinator.rs:178-215).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mrgpu.h"

static unsigned char *read_file(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *b = (unsigned char *)malloc((size_t)sz + 1);
    if (sz > 0 && fread(b, 1, (size_t)sz, f) != (size_t)sz) {
        fclose(f);
        free(b);
        return NULL;
    }
    fclose(f);
    *n = (size_t)sz;
    return b;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: worker_harness <map_n> <reduce_n> [--indexer]\n");
        return 2;
    }
    const int map_n = atoi(argv[1]);
    const unsigned reduce_n = (unsigned)atoi(argv[2]);
    const int app = (argc > 3 && !strcmp(argv[3], "--indexer")) ? MRG_APP_INDEXER : MRG_APP_WC;
    mrg_ctx *ctx = NULL;
    if (mrg_open(0, &ctx) != MRG_OK) {
        fprintf(stderr, "mrg_open: %s\n", mrg_last_error());
        return 1;
    }
    mrg_parts **parts = (mrg_parts **)calloc((size_t)map_n + 1, sizeof(mrg_parts *));
    char **names = (char **)calloc((size_t)map_n + 1, sizeof(char *));
    int rc = 0;
    for (int m = 0; m < map_n && !rc; ++m) {
        names[m] = (char *)malloc(64);
        snprintf(names[m], 64, "data/gut-%d.txt", m);  /* worker.rs:67 */
        size_t n = 0;
        unsigned char *bytes = read_file(names[m], &n);
        if (!bytes) {
            fprintf(stderr, "cannot read %s\n", names[m]);
            rc = 1;
            break;
        }
        if (mrg_map(ctx, app, bytes, n, names[m], (uint32_t)m, reduce_n, 0, &parts[m]) != MRG_OK) {
            fprintf(stderr, "mrg_map(%d): %s\n", m, mrg_last_error());
            rc = 1;
        }
        free(bytes);
    }
    for (unsigned r = 0; r < reduce_n && !rc; ++r) {
        uint8_t *out = NULL;
        size_t len = 0;
        if (mrg_reduce(ctx, app, r, (const mrg_parts *const *)parts, (size_t)map_n, reduce_n, 0,
                       (const char *const *)names, (uint32_t)map_n, &out, &len) != MRG_OK) {
            fprintf(stderr, "mrg_reduce(%u): %s\n", r, mrg_last_error());
            rc = 1;
            break;
        }
        char path[64];
        snprintf(path, sizeof path, "mr-%u.txt", r);
        FILE *f = fopen(path, "wb");
        if (!f || (len && fwrite(out, 1, len, f) != len)) rc = 1;
        if (f) fclose(f);
        mrg_free(out);
    }
    for (int m = 0; m < map_n; ++m) {
        if (parts[m]) mrg_parts_free(parts[m]);
        free(names[m]);
    }
    free(parts);
    free(names);
    mrg_close(ctx);
    return rc;
}
