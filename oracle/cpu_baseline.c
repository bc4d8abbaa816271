/*
 * cpu_baseline.c -- TEST/BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * Times the host-CPU path the reference actually runs for each request
 * signature: libsodium's Ed25519 verify (stp_core/crypto/nacl_wrappers.py:108
 * -> libnacl.crypto_sign_open -> crypto_sign_verify_detached), one pthread per
 * host core, over the same packed inputs the GPU receives
 * (include/edverify.h layout: sig64[n*64], pk32[n*32], msgs + msg_off[n+1]).
 *
 * libsodium is dlopen()ed (never linked), so this file builds on any box; if
 * it is not loadable the harness times the plain-C oracle restatement instead
 * and reports kind = "port".
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

int oracle_verify_detached(const uint8_t sig[64], const uint8_t *m, uint64_t mlen, const uint8_t pk[32]);

typedef int (*verify_fn)(const unsigned char *, const unsigned char *, unsigned long long, const unsigned char *);
typedef int (*init_fn)(void);
typedef const char *(*version_fn)(void);

static verify_fn g_sodium_verify = NULL;
static char g_version[64] = "";

static int load_sodium(void) {
  if (g_sodium_verify) return 1;
  const char *cands[] = {"libsodium.so.23", "/opt/conda/lib/libsodium.so.23", "libsodium.so", "/opt/conda/lib/libsodium.so", NULL};
  for (int i = 0; cands[i]; i++) {
    void *h = dlopen(cands[i], RTLD_NOW | RTLD_LOCAL);
    if (!h) continue;
    init_fn in = (init_fn)dlsym(h, "sodium_init");
    verify_fn v = (verify_fn)dlsym(h, "crypto_sign_verify_detached");
    version_fn ver = (version_fn)dlsym(h, "sodium_version_string");
    if (!in || !v) continue;
    if (in() < 0) continue;
    g_sodium_verify = v;
    if (ver) snprintf(g_version, sizeof g_version, "%s", ver());
    return 1;
  }
  return 0;
}

/* Returns the libsodium version string, or "" when libsodium is absent. */
const char *cpu_baseline_sodium_version(void) {
  load_sodium();
  return g_version;
}

typedef struct {
  const uint8_t *sig, *pk, *msgs;
  const uint64_t *off;
  const uint64_t *start, *end; /* spans form (off == NULL): item i's message is msgs[start[i], end[i]) */
  uint64_t lo, hi;
  int use_sodium;
  uint8_t *ok; /* one byte per item */
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint64_t a = j->off ? j->off[i] : j->start[i], b = j->off ? j->off[i + 1] : j->end[i];
    const uint8_t *m = j->msgs + a;
    uint64_t ml = b - a;
    int r = j->use_sodium ? g_sodium_verify(j->sig + 64 * i, m, ml, j->pk + 32 * i)
                          : oracle_verify_detached(j->sig + 64 * i, m, ml, j->pk + 32 * i);
    j->ok[i] = (r == 0);
  }
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* Verify n items on `threads` threads.  use_sodium: 1 = libsodium (falls back
 * to the oracle, returning kind 0, if absent), 0 = oracle restatement.
 * Writes one verdict byte per item into ok[n] and the wall seconds into
 * *seconds.  Returns 1 if libsodium was timed, 0 if the oracle was, -1 on error. */
int cpu_baseline_run(const uint8_t *sig64, const uint8_t *pk32, const uint8_t *msgs, const uint64_t *msg_off, uint64_t n,
                     int threads, int use_sodium, uint8_t *ok, double *seconds) {
  if (threads < 1 || threads > 1024) return -1;
  int sodium = use_sodium && load_sodium();
  pthread_t tid[1024];
  job_t jobs[1024];
  double t0 = now_s();
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){sig64, pk32, msgs, msg_off, NULL, NULL, n * t / threads, n * (t + 1) / threads, sodium, ok};
    if (pthread_create(&tid[t], NULL, worker, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  *seconds = now_s() - t0;
  return sodium;
}

/* Verdicts of n items whose messages are spans msgs[start[i], end[i]) (several
 * items may share one message: configs[3]'s multi-signature requests), on
 * `threads` threads -- the parity tests' full-batch check against libsodium.
 * Returns 1 if libsodium gave the verdicts, 0 if it is absent (nothing
 * written), -1 on error. */
int cpu_baseline_verdicts_spans(const uint8_t *sig64, const uint8_t *pk32, const uint8_t *msgs, const uint64_t *start,
                                const uint64_t *end, uint64_t n, int threads, uint8_t *ok) {
  if (threads < 1 || threads > 1024) return -1;
  if (!load_sodium()) return 0;
  pthread_t tid[1024];
  job_t jobs[1024];
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){sig64, pk32, msgs, NULL, start, end, n * t / threads, n * (t + 1) / threads, 1, ok};
    if (pthread_create(&tid[t], NULL, worker, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  return 1;
}
