/* TEST INFRASTRUCTURE ONLY: drives the oracle under -fsanitize=address,undefined (make -C oracle check-asan). */
#include <stdio.h>
#include <stdlib.h>
#include "oracle.h"

int main(void) {
    gso_ds* a = gso_ds_new();
    gso_ds* b = gso_ds_new();
    for (int i = 0; i < 8; ++i) gso_ds_union(a, i, i + 2);
    for (int i = 0; i < 8; ++i) gso_ds_union(b, i, i + 100);
    gso_ds_merge(b, a);
    int64_t r;
    if (gso_ds_size(b) != 18 || !gso_ds_find(b, 5, &r) || gso_ds_find(b, 12345, &r)) return 1;
    gso_ds* keep = gso_combine(a, b);
    gso_ds_free(keep == a ? b : a);
    gso_ds_free(keep);
    const uint64_t n = 200000;
    int64_t* s = malloc(n * sizeof(int64_t));
    int64_t* d = malloc(n * sizeof(int64_t));
    gso_gen_rmat(s, d, 0, n, 14, 3, 2448131358u, 816043786u, 816043786u, 1);
    gso_run_cfg cfg = {4096, 4, 4, GSO_EMIT_DENSE, 1 << 14};
    uint64_t nw = (n + 4095) / 4096;
    uint64_t* sums = malloc(nw * sizeof(uint64_t));
    int64_t* labels = malloc(nw * (1 << 14) * sizeof(int64_t));
    int64_t* fin = malloc((1 << 14) * sizeof(int64_t));
    gso_run_stats st;
    if (gso_cc_run(s, d, n, &cfg, sums, labels, fin, &st)) return 1;
    gso_gen_er(s, d, 7, n, 1 << 14, 2);
    cfg.emit_mode = GSO_EMIT_FLATTEN;
    if (gso_cc_run(s, d, n, &cfg, NULL, NULL, NULL, &st)) return 1;
    printf("oracle sanitizer run OK: %llu windows, %llu vertices\n", (unsigned long long)st.windows,
           (unsigned long long)st.final_vertices);
    free(s); free(d); free(sums); free(labels); free(fin);
    return 0;
}
