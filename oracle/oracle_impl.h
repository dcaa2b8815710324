/*
 * oracle_impl.h -- body of the CPU restatement, instantiated by rnnt_oracle.c once with
 * REAL=double (the parity golden) and once with REAL=float (mirrors cpu_rnnt.h<float> rounding).
 *
 * TEST INFRASTRUCTURE ONLY: this is the checker, never the product. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Every function cites the reference lines it restates (paths relative to the reference repo).
 */

/* rnnt_helper.h:16-30 -- log_sum_exp with -inf short-circuit.  The reference calls the unqualified
 * C functions exp()/log1p() on a (b - a) computed in REAL, i.e. the transcendental runs in double
 * and the result is rounded back to REAL; we mirror that exactly. */
static REAL SFX(lse)(REAL a, REAL b) {
    if (a == -(REAL)INFINITY) return b;
    if (b == -(REAL)INFINITY) return a;
    if (a > b) {
        REAL d = b - a;
        return (REAL)(log1p(exp((double)d)) + (double)a);
    } else {
        REAL d = a - b;
        return (REAL)(log1p(exp((double)d)) + (double)b);
    }
}

/* std::exp(float) in cpu_rnnt.h:219-233 is the float overload; expf here. */
static REAL SFX(gexp)(REAL x) { return (sizeof(REAL) == sizeof(float)) ? (REAL)expf((float)x) : (REAL)exp((double)x); }

typedef struct {
    int T, S, V;
    const float *acts;   /* utterance base: row (t,s) at acts + (t*(S+1)+s)*V */
    const int *labels;   /* utterance label row */
    const int *min_s;    /* [T] */
    const int *max_s;    /* [T] */
    REAL *denom;         /* [T*(S+1)] */
    REAL *alpha;         /* [T*(S+1)] dense (the reference packs the band; values identical) */
    REAL *beta;          /* [T*(S+1)] */
} SFX(utt_t);

static inline REAL SFX(act)(const SFX(utt_t) *u, int t, int s, int v) {
    /* cpu_workspace_manager.h:125-135 (act_index), widened to 64-bit offsets */
    return (REAL)u->acts[((int64_t)t * (u->S + 1) + s) * (int64_t)u->V + v];
}

/* cpu_workspace_manager.h:161-181 */
static REAL SFX(get_alpha)(const SFX(utt_t) *u, int t, int s) {
    if (s == -1) return -(REAL)INFINITY;
    if (t == -1) return s == 0 ? (REAL)0 : -(REAL)INFINITY;
    if (s < u->min_s[t] || s > u->max_s[t]) return -(REAL)INFINITY;
    if (s > t + 1 || u->S - s > u->T - 1 - t) return -(REAL)INFINITY;
    return u->alpha[(int64_t)t * (u->S + 1) + s];
}

/* cpu_workspace_manager.h:185-205 */
static REAL SFX(get_beta)(const SFX(utt_t) *u, int t, int s) {
    if (s == u->S + 1) return -(REAL)INFINITY;
    if (t == u->T) return s == u->S ? (REAL)0 : -(REAL)INFINITY;
    if (t > 0 && (s < u->min_s[t - 1] || s > u->max_s[t - 1])) return -(REAL)INFINITY;
    if (s > t || u->S - s - 1 > u->T - 1 - t) return -(REAL)INFINITY;
    return u->beta[(int64_t)t * (u->S + 1) + s];
}

static inline REAL SFX(den)(const SFX(utt_t) *u, int t, int s) { return u->denom[(int64_t)t * (u->S + 1) + s]; }

static inline int SFX(maxi)(int a, int b) { return a > b ? a : b; }
static inline int SFX(mini)(int a, int b) { return a < b ? a : b; }

/* cpu_rnnt.h:98-115 -- per-row log-softmax denominator, sequential LSE over v (all rows). Frames run in
 * parallel when the utterance loop is not (one utterance per call): rows are independent, so this changes
 * nothing but the wall time. */
static void SFX(denoms)(SFX(utt_t) *u) {
#pragma omp parallel for schedule(static)
    for (int t = 0; t < u->T; ++t) {
        for (int s = 0; s <= u->S; ++s) {
            REAL max_v = -(REAL)INFINITY;
            for (int v = 0; v < u->V; ++v) {
                REAL a = SFX(act)(u, t, s, v);
                max_v = (max_v < a) ? a : max_v; /* std::max */
            }
            REAL d = -(REAL)INFINITY;
            for (int v = 0; v < u->V; ++v) d = SFX(lse)(d, SFX(act)(u, t, s, v) - max_v);
            u->denom[(int64_t)t * (u->S + 1) + s] = -max_v - d;
        }
    }
}

/* cpu_rnnt.h:155-183 ; band limits cpu_workspace_manager.h:67-72 */
static REAL SFX(alphas)(SFX(utt_t) *u, int blank) {
    const int T = u->T, S = u->S;
    for (int t = 0; t < T; ++t) {
        int lo = SFX(maxi)(u->min_s[t], t - (T - 1 - S));
        int hi = SFX(mini)(SFX(mini)(u->max_s[t], t + 1), S); /* clamp to S: see DESIGN.md (reference UB) */
        for (int s = lo; s <= hi; ++s) {
            REAL no_emit = SFX(get_alpha)(u, t - 1, s) + SFX(act)(u, t, s, blank) + SFX(den)(u, t, s);
            REAL emit = SFX(get_alpha)(u, t - 1, s - 1);
            if (s > 0) emit += SFX(act)(u, t, s - 1, u->labels[s - 1]) + SFX(den)(u, t, s - 1);
            u->alpha[(int64_t)t * (S + 1) + s] = SFX(lse)(emit, no_emit);
        }
    }
    return SFX(get_alpha)(u, T - 1, S);
}

/* cpu_rnnt.h:185-214 ; band limits cpu_workspace_manager.h:74-86 */
static REAL SFX(betas)(SFX(utt_t) *u, int blank) {
    const int T = u->T, S = u->S;
    for (int t = T - 1; t >= 0; --t) {
        int lo = t == 0 ? 0 : SFX(maxi)(u->min_s[t - 1], t - (T - S));
        int hi = t == 0 ? 0 : SFX(mini)(u->max_s[t - 1], t);
        for (int s = lo; s <= hi; ++s) {
            REAL no_emit = SFX(get_beta)(u, t + 1, s) + SFX(act)(u, t, s, blank) + SFX(den)(u, t, s);
            REAL emit = SFX(get_beta)(u, t + 1, s + 1);
            if (s < S) emit += SFX(act)(u, t, s, u->labels[s]) + SFX(den)(u, t, s);
            u->beta[(int64_t)t * (S + 1) + s] = SFX(lse)(emit, no_emit);
        }
    }
    return SFX(get_beta)(u, 0, 0);
}

/* cpu_rnnt.h:216-236 -- gradient w.r.t. every logit of the utterance (out-of-band rows -> 0); frames in
 * parallel as in denoms(). */
static void SFX(grads)(const SFX(utt_t) *u, REAL ll, int blank, REAL *g) {
    const int T = u->T, S = u->S, V = u->V;
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; ++t) {
        for (int s = 0; s <= S; ++s) {
            REAL a = SFX(get_alpha)(u, t - 1, s);
            REAL b0 = SFX(get_beta)(u, t, s);
            REAL b1 = SFX(get_beta)(u, t + 1, s);
            REAL b2 = SFX(get_beta)(u, t + 1, s + 1);
            REAL dn = SFX(den)(u, t, s);
            int lab = s < S ? u->labels[s] : -1;
            REAL *row = g + ((int64_t)t * (S + 1) + s) * V;
            for (int v = 0; v < V; ++v) {
                REAL x = SFX(act)(u, t, s, v);
                REAL gv = SFX(gexp)(x + dn - ll + a + b0);
                if (v == blank) {
                    gv -= SFX(gexp)(x + dn - ll + a + b1);
                } else if (s < S && v == lab) {
                    gv -= SFX(gexp)(x + dn - ll + a + b2);
                }
                row[v] = gv;
            }
        }
    }
}

/* Full entry: cpu_rnnt.h:42-66 (cost_and_grad) / :68-92 (cost, when grads == NULL);
 * validation cpu_workspace_manager.h:99-107; alignment band cpu_workspace_manager.h:207-224. */
int SFX(mrnnt_oracle)(const float *acts, const int *labels, int64_t label_stride, int B, const int *T, const int *S,
                      int V, int blank, const int *alignment, int64_t align_stride, int max_shift, int align_blank,
                      REAL *costs, REAL *grads, REAL *denom_out, REAL *alpha_out, REAL *beta_out, int num_threads) {
    if (B <= 0 || V <= 0) return 2;
    for (int b = 0; b < B; ++b)
        if (T[b] <= 0 || S[b] < 0 || T[b] < S[b]) return 2;

    int64_t *row_off = (int64_t *)malloc(sizeof(int64_t) * (B + 1));
    row_off[0] = 0;
    for (int b = 0; b < B; ++b) row_off[b + 1] = row_off[b] + (int64_t)T[b] * (S[b] + 1);

#ifdef _OPENMP
    if (num_threads > 0) omp_set_num_threads(num_threads);
#else
    (void)num_threads;
#endif
    int err = 0;
    /* utterances in parallel; a single utterance instead parallelises its frames (the nested regions in
     * denoms() / grads() are active only when this one is not) */
#pragma omp parallel for schedule(dynamic, 1) if (B > 1)
    for (int b = 0; b < B; ++b) {
        const int Tb = T[b], Sb = S[b];
        const int64_t nrow = (int64_t)Tb * (Sb + 1);
        SFX(utt_t) u;
        u.T = Tb;
        u.S = Sb;
        u.V = V;
        u.acts = acts + row_off[b] * (int64_t)V;
        u.labels = labels + (int64_t)b * label_stride;
        int *mins = (int *)malloc(sizeof(int) * Tb);
        int *maxs = (int *)malloc(sizeof(int) * Tb);
        REAL *buf = (REAL *)malloc(sizeof(REAL) * 3 * nrow);
        if (!mins || !maxs || !buf) {
            err = 1;
            free(mins);
            free(maxs);
            free(buf);
            continue;
        }
        for (int t = 0; t < Tb; ++t) {
            mins[t] = 0;
            maxs[t] = Sb;
        }
        if (alignment) { /* cpu_workspace_manager.h:207-224 */
            int *m = (int *)malloc(sizeof(int) * (Tb + 1));
            m[0] = 0;
            for (int t = 0; t < Tb; ++t) m[t + 1] = m[t] + (alignment[(int64_t)b * align_stride + t] == align_blank ? 0 : 1);
            for (int t = 0; t < Tb; ++t) {
                mins[t] = m[SFX(maxi)(0, t + 1 - max_shift)];
                maxs[t] = m[SFX(mini)(Tb, t + 1 + max_shift)];
            }
            free(m);
        }
        u.min_s = mins;
        u.max_s = maxs;
        u.denom = buf;
        u.alpha = buf + nrow;
        u.beta = buf + 2 * nrow;
        for (int64_t i = 0; i < 3 * nrow; ++i) buf[i] = -(REAL)INFINITY;

        SFX(denoms)(&u);
        REAL ll = SFX(alphas)(&u, blank);
        if (grads) {
            (void)SFX(betas)(&u, blank); /* cpu_rnnt.h:254-263; fwd/bwd mismatch only warns there */
            SFX(grads)(&u, ll, blank, grads + row_off[b] * (int64_t)V);
        }
        costs[b] = -ll;

        /* debug/inspection outputs: getter values (incl. virtual -inf) in the dense [rows] layout */
        for (int t = 0; t < Tb; ++t)
            for (int s = 0; s <= Sb; ++s) {
                int64_t r = row_off[b] + (int64_t)t * (Sb + 1) + s;
                if (denom_out) denom_out[r] = SFX(den)(&u, t, s);
                if (alpha_out) alpha_out[r] = SFX(get_alpha)(&u, t, s);
                if (beta_out) beta_out[r] = grads ? SFX(get_beta)(&u, t, s) : -(REAL)INFINITY;
            }
        free(mins);
        free(maxs);
        free(buf);
    }
    free(row_off);
    return err ? 1 : 0;
}
