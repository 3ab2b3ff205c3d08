/* Descent-walk lengths of the hull SDF (CPU study; tools/walk_study.py).
 * Compiles the oracle with a hook that records, per (point, hull) evaluation,
 * the number of accepted walk steps and whether the exhaustive scan ran.
 * Study only: never loaded by the product, the tests or the bench. */
static __thread int g_walk_steps, g_walk_scan;
#define ORACLE_WALK_HOOK(steps, scan) (g_walk_steps = (steps), g_walk_scan = (scan))
#include "../oracle/flash_oracle.c"

/* for each (point i, hull k) of the pairs given: d and the walk length (-1:
 * no walk — inside, or the projection fell inside the max face) */
void walk_study(const oracle_posed* m, const double* pts, const int32_t* pi, const int32_t* hk, int64_t npairs,
                double* d_out, int32_t* steps_out, int32_t* scan_out) {
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t j = 0; j < npairs; ++j) {
    double d, g[3];
    g_walk_steps = -1;
    g_walk_scan = 0;
    oracle_hull_sdf(m, hk[j], pts + 3 * (int64_t)pi[j], &d, g);
    d_out[j] = d;
    steps_out[j] = g_walk_steps;
    scan_out[j] = g_walk_scan;
  }
}
