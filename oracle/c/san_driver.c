/* TEST INFRASTRUCTURE ONLY (oracle/): a stand-alone driver that runs the C oracle's entry points
 * (bls_oracle.c) in a process of its own, so the oracle can be built with
 * -fsanitize=address,undefined (Makefile target `san`) and exercised on the golden fixtures without
 * loading a sanitizer runtime into Python (tests/test_sanitizers.py).
 *
 *   san_driver <op> <in> <out>
 *
 * <in>: the op's arguments in order, each a blob (u64 little-endian length, then the bytes); integer
 * arguments are 8-byte little-endian blobs.  Every blob is copied into a heap block of exactly its
 * length, so an oracle read past an argument is a heap-buffer-overflow report.  <out>: the op's output
 * buffers, concatenated, then the 4-byte return code. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oc_verify_batch(int mode, size_t n, size_t q, const uint8_t* s1, const uint8_t* s2, const uint8_t* msgs,
                    const uint8_t* X, const uint8_t* Y, int per_cred_vk, const uint8_t* gtilde, uint8_t* verdicts,
                    uint8_t* gts, int nthreads);
int oc_pairing(const uint8_t* Pb, const uint8_t* Qb, uint8_t* gt_out);
int oc_gen_mul_mt(int group, size_t n, const uint8_t* ks, uint8_t* out, int nthreads);
int oc_lagrange(size_t t, const uint64_t* ids, uint8_t* out);
int oc_signature_aggregate(int mode, size_t len, size_t t, const uint64_t* ids, const uint8_t* s1, const uint8_t* s2,
                           uint8_t* out_s1, uint8_t* out_s2);
int oc_verkey_aggregate(int mode, size_t len, size_t t, size_t q, const uint64_t* ids, const uint8_t* X,
                        const uint8_t* Y, uint8_t* outX, uint8_t* outY);
int oc_pok_verify(int mode, size_t q, size_t r, const uint8_t* s1b, const uint8_t* s2b, const uint8_t* Jb,
                  const uint8_t* Tb, const uint8_t* responses, size_t nresp, const uint8_t* chal,
                  const uint64_t* revealed_idx, const uint8_t* revealed_msgs, const uint8_t* Xb, const uint8_t* Yb,
                  const uint8_t* gtb, uint8_t* gt_out);

#define MAXARG 32
static uint8_t* arg[MAXARG];
static uint64_t alen[MAXARG];
static int nargs;

static int load(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    for (nargs = 0; nargs < MAXARG; nargs++) {
        uint64_t len;
        if (fread(&len, 8, 1, f) != 1) break;
        arg[nargs] = (uint8_t*)malloc(len ? len : 1);
        alen[nargs] = len;
        if (len && fread(arg[nargs], 1, len, f) != len) {
            fclose(f);
            return -1;
        }
    }
    fclose(f);
    return 0;
}
static uint64_t u(int k) {
    uint64_t v = 0;
    memcpy(&v, arg[k], alen[k] < 8 ? alen[k] : 8);
    return v;
}
static uint8_t* out_buf(size_t len) { return (uint8_t*)calloc(len ? len : 1, 1); }

int main(int argc, char** argv) {
    if (argc != 4 || load(argv[2])) {
        fprintf(stderr, "usage: san_driver <op> <in> <out>\n");
        return 2;
    }
    const char* op = argv[1];
    uint8_t* o1 = NULL;
    uint8_t* o2 = NULL;
    size_t l1 = 0, l2 = 0;
    int rc = -100;
    if (!strcmp(op, "verify") && nargs == 12) {
        /* mode n q s1 s2 msgs X Y per g nthreads want_gt */
        const size_t n = u(1);
        l1 = n;
        l2 = u(11) ? 576 * n : 0;
        o1 = out_buf(l1);
        o2 = l2 ? out_buf(l2) : NULL;
        rc = oc_verify_batch((int)u(0), n, u(2), arg[3], arg[4], arg[5], arg[6], arg[7], (int)u(8), arg[9], o1, o2,
                             (int)u(10));
    } else if (!strcmp(op, "gen_mul") && nargs == 3) {
        /* group n ks (4 threads) */
        l1 = u(1) * (u(0) == 1 ? 97 : 192);
        o1 = out_buf(l1);
        rc = oc_gen_mul_mt((int)u(0), u(1), arg[2], o1, 4);
    } else if (!strcmp(op, "pairing") && nargs == 2) {
        l1 = 576;
        o1 = out_buf(l1);
        rc = oc_pairing(arg[0], arg[1], o1);
    } else if (!strcmp(op, "lagrange") && nargs == 2) {
        l1 = 48 * u(0);
        o1 = out_buf(l1);
        rc = oc_lagrange(u(0), (const uint64_t*)arg[1], o1);
    } else if (!strcmp(op, "sigagg") && nargs == 7) {
        /* mode len t ids s1 s2 sb */
        l1 = l2 = u(6);
        o1 = out_buf(l1);
        o2 = out_buf(l2);
        rc = oc_signature_aggregate((int)u(0), u(1), u(2), (const uint64_t*)arg[3], arg[4], arg[5], o1, o2);
    } else if (!strcmp(op, "vkagg") && nargs == 8) {
        /* mode len t q ids X Y ob */
        l1 = u(7);
        l2 = u(7) * u(3);
        o1 = out_buf(l1);
        o2 = out_buf(l2);
        rc = oc_verkey_aggregate((int)u(0), u(1), u(2), u(3), (const uint64_t*)arg[4], arg[5], arg[6], o1, o2);
    } else if (!strcmp(op, "pok") && nargs == 15) {
        /* mode q r s1 s2 J T resp nresp chal idx rev_msgs X Y g */
        l1 = 576;
        o1 = out_buf(l1);
        rc = oc_pok_verify((int)u(0), u(1), u(2), arg[3], arg[4], arg[5], arg[6], arg[7], u(8), arg[9],
                           (const uint64_t*)arg[10], arg[11], arg[12], arg[13], arg[14], o1);
    } else {
        fprintf(stderr, "san_driver: unknown op %s or wrong argument count %d\n", op, nargs);
        return 2;
    }
    FILE* f = fopen(argv[3], "wb");
    if (!f) return 2;
    if (l1) fwrite(o1, 1, l1, f);
    if (l2) fwrite(o2, 1, l2, f);
    int32_t r32 = rc;
    fwrite(&r32, 4, 1, f);
    fclose(f);
    free(o1);
    free(o2);
    for (int k = 0; k < nargs; k++) free(arg[k]);
    return 0;
}
