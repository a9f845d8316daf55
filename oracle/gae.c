/* CPU oracle — TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 *
 * Plain-C restatement of the reference's Cython GAE, /root/reference/puffer_phc/c_gae.pyx:11-32:
 * a backward pass over the flat env-sorted buffer, float32 throughout, A[n-1] = 0,
 *   nnt   = 1 - done[t+1]
 *   delta = r[t+1] + gamma * v[t+1] * nnt - v[t]
 *   A[t]  = delta + gamma * lambda * nnt * A[t+1]
 * Built with -ffp-contract=off so every product / sum rounds separately, as Cython's generated C
 * does on x86-64 (SSE float arithmetic, no FMA).  Pinned by tests/golden/gae.npz (generated from
 * the reference's own c_gae.pyx) in tests/test_oracle_golden.py. */
#include <stdint.h>

void phc_oracle_gae(const float *dones, const float *values, const float *rewards, int64_t n, float gamma,
                    float gae_lambda, float *advantages) {
  if (n <= 0) return;
  float last = 0.0f;
  advantages[n - 1] = 0.0f;
  for (int64_t t = 0; t < n - 1; ++t) {
    const int64_t cur = n - 2 - t, nxt = n - 1 - t;
    const float nnt = 1.0f - dones[nxt];
    const float delta = rewards[nxt] + gamma * values[nxt] * nnt - values[cur];
    last = delta + gamma * gae_lambda * nnt * last;
    advantages[cur] = last;
  }
}
