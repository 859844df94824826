/*
 * gotorch_cpu.c — C restatement of the reference's Go CPU path for BASELINE
 * configs[0]: gotorch.AffineLayer.Forward (go/gotorch/layers.go:57-70) over
 * gotorch.MatMul (go/gotorch/ops.go:15-34) and matmulParallel (ops.go:49-81).
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY: loaded by tests/ and the cpu_baseline leg
 * of bench.py. It is a restatement, not Go (no Go toolchain in this image): the
 * same float64 arithmetic in the same order, the same work split.
 *   Forward: inputCache = input.Clone(); out = MatMul(input, W); out[i][j] += b[j]
 *   MatMul: M*N*K > 10000 -> matmulParallel, else matmulNaive; both compute
 *           c[i][j] = sum_k a[i][k] * b[k][j] with the k loop innermost (B read
 *           with stride N), starting from sum = 0.0
 *   matmulParallel: numWorkers = runtime.NumCPU() (here: `workers`), capped at M;
 *           rowsPerWorker = ceil(M / numWorkers); worker w takes rows
 *           [w*rpw, min((w+1)*rpw, M)) — one goroutine each, then wg.Wait()
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    const double *a, *b;
    double *c;
    int K, N, start, end;
} GtRows;

/* the goroutine body of matmulParallel (ops.go:65-76) */
static void *gt_rows(void *p) {
    const GtRows *r = (const GtRows *)p;
    for (int i = r->start; i < r->end; i++)
        for (int j = 0; j < r->N; j++) {
            double sum = 0.0;
            for (int k = 0; k < r->K; k++) sum += r->a[(long)i * r->K + k] * r->b[(long)k * r->N + j];
            r->c[(long)i * r->N + j] = sum;
        }
    return NULL;
}

/* gotorch.MatMul (ops.go:15-34); c is M x N, overwritten */
void gt_matmul(const double *a, const double *b, double *c, int M, int K, int N, int workers) {
    if ((long long)M * N * K > 10000) {
        int nw = workers < 1 ? 1 : workers;
        if (nw > M) nw = M;
        const int rpw = (M + nw - 1) / nw;
        pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nw);
        GtRows *args = (GtRows *)malloc(sizeof(GtRows) * nw);
        int started = 0;
        for (int w = 0; w < nw; w++) {
            int s = w * rpw, e = s + rpw;
            if (e > M) e = M;
            GtRows r = {a, b, c, K, N, s, e};
            args[w] = r;
            /* Go starts the goroutine even for an empty range (s >= M); it does nothing */
            if (s >= e) continue;
            if (pthread_create(&th[started], NULL, gt_rows, &args[w]) == 0)
                started++;
            else
                gt_rows(&args[w]);
        }
        for (int w = 0; w < started; w++) pthread_join(th[w], NULL);
        free(th);
        free(args);
    } else {
        GtRows r = {a, b, c, K, N, 0, M};  /* matmulNaive (ops.go:36-47): same loop order */
        gt_rows(&r);
    }
}

/* AffineLayer.Forward (layers.go:57-70): x [M x K] -> y [M x N]; cache receives the
 * input clone (l.inputCache = input.Clone()) */
void gt_affine_forward(const double *x, int M, int K, const double *W, const double *bias, int N, double *y,
                       double *cache, int workers) {
    memcpy(cache, x, sizeof(double) * (size_t)M * K);
    memset(y, 0, sizeof(double) * (size_t)M * N);  /* c := Zeros([]int{M, N}) (ops.go:26) */
    gt_matmul(x, W, y, M, K, N, workers);
    for (int i = 0; i < M; i++)
        for (int j = 0; j < N; j++) y[(long)i * N + j] += bias[j];
}
