/*
 * crlot_oracle.c -- CPU restatement of crlot-dsp's STFT->OLA hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see crlot_oracle.h).  Compiled with
 * -ffp-contract=off so every float operation rounds exactly as written; the
 * FMA-shaped steps of the reference (std::fma in kernels.cc:18-36) use fmaf.
 *
 * Each function cites the reference file:line it restates.  kissfft 131.1.0
 * (third-party, absent: /root/reference/third_party/kissfft is an empty
 * submodule; version pinned by /root/reference/Makefile:17) is restated from
 * its published algorithm: kf_factor, kf_work, kf_bfly2/3/4/5/generic,
 * kiss_fftr / kiss_fftri with super-twiddles, twiddles = (float)cos/sin(double).
 */
#define _GNU_SOURCE
#include "crlot_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ======================================================================== */
/* WindowLUT (dsp/window/WindowLUT.cc)                                      */
/* ======================================================================== */

/* WindowLUT::calculateSum / calculateSumOfSquares (WindowLUT.cc:170-193) */
static double win_sum(const float* w, size_t n) {
    double s = 0.0;
    for (size_t i = 0; i < n; ++i) s += (double)w[i];
    return s;
}
static double win_sumsq(const float* w, size_t n) {
    double s = 0.0;
    for (size_t i = 0; i < n; ++i) {
        double v = (double)w[i];
        s += v * v;
    }
    return s;
}

/* WindowLUT::applyNormalization (WindowLUT.cc:317-388); hop_size defaults to 0
 * in createWindow's call (WindowLUT.cc:250), so OLA_SUM_WSQ takes the L2 branch. */
static void win_normalize(float* w, size_t n, int norm) {
    switch (norm) {
        case OR_NORM_SUM_TO_ONE: {
            double s = win_sum(w, n);
            if (s > 0.0) {
                float sc = (float)(1.0 / s);
                for (size_t i = 0; i < n; ++i) w[i] *= sc;
            }
            break;
        }
        case OR_NORM_L2:
        case OR_NORM_OLA_UNITY_GAIN:
        case OR_NORM_OLA_SUM_WSQ: {
            double s = win_sumsq(w, n);
            if (s > 0.0) {
                float sc = (float)(1.0 / sqrt(s));
                for (size_t i = 0; i < n; ++i) w[i] *= sc;
            }
            break;
        }
        default:
            break;
    }
}

/* WindowLUT::createWindow + generate*Window (WindowLUT.cc:215-315) */
int or_window(int type, size_t n, int periodic, int norm, float* out) {
    if (n == 0) return -1;
    if (type == OR_BLACKMAN_HARRIS || type < 0 || type > OR_BLACKMAN_HARRIS) return -2;
    if (type == OR_RECT) {
        for (size_t i = 0; i < n; ++i) out[i] = 1.0f;
    } else if (n == 1) {
        out[0] = 1.0f;
    } else {
        const double pi = M_PI;
        const double den = periodic ? (double)n : (double)(n - 1);
        const double factor = 2.0 * pi / den;
        for (size_t i = 0; i < n; ++i) {
            double angle = factor * (double)i;
            if (type == OR_HANN) {
                out[i] = (float)(0.5 * (1.0 - cos(angle)));
            } else if (type == OR_HAMMING) {
                out[i] = (float)(0.54 - 0.46 * cos(angle));
            } else { /* BLACKMAN */
                double c1 = cos(angle);
                double c2 = cos(2.0 * angle);
                out[i] = (float)(0.42 - 0.5 * c1 + 0.08 * c2);
            }
        }
    }
    if (norm != OR_NORM_NONE) win_normalize(out, n, norm);
    return 0;
}

/* ======================================================================== */
/* COLA norm (OLAAccumulator.cc:249-288, norm_builder.cc:8-52)              */
/* ======================================================================== */

size_t or_ring_len(size_t frame_size, size_t hop) {
    size_t min_overlaps = (frame_size + hop - 1) / hop; /* :251 */
    return (min_overlaps + 20) * hop;                   /* :254-257 */
}

void or_build_norm_linear(float* norm, const float* window, size_t ring_len, size_t n,
                          size_t h) {
    for (size_t i = 0; i < ring_len; ++i) norm[i] = 0.0f; /* :11 */
    if (ring_len == 0 || n == 0 || h == 0) return;
    const int64_t R = (int64_t)ring_len;
    /* floor_div(-N, H) (:35) and K_end (:37) */
    const int64_t a = -(int64_t)n;
    const int64_t k_start = (a - (int64_t)h + 1) / (int64_t)h;
    const int64_t k_end = (R + (int64_t)n - 1 + (int64_t)h - 1) / (int64_t)h;
    for (int64_t k = k_start; k <= k_end; ++k) {
        int64_t s = k * (int64_t)h;
        /* split_span (:20-31): negative start -> R + (s % R) */
        if (s < 0) {
            s = R + (s % R);
            if (s < 0) s += R;
        }
        size_t st = (size_t)(s % R);
        size_t first = n < ring_len - st ? n : ring_len - st;
        size_t second = n - first;
        for (size_t i = 0; i < first; ++i) norm[st + i] += window[i];       /* :44-45 */
        for (size_t i = 0; i < second; ++i) norm[i] += window[first + i];   /* :48-49 */
    }
}

void or_init_normalization(float* norm, const float* window, size_t ring_len, size_t n, size_t h,
                           int apply_window_inside, float eps) {
    if (window == NULL || !apply_window_inside) { /* :261-272 */
        for (size_t i = 0; i < ring_len; ++i) norm[i] = 1.0f;
        return;
    }
    if (h == n) { /* :275-282 */
        for (size_t i = 0; i < ring_len; ++i) {
            float w = window[i % n];
            norm[i] = w > eps ? w : eps; /* std::max(window, eps) */
        }
        return;
    }
    or_build_norm_linear(norm, window, ring_len, n, h);
}

/* ======================================================================== */
/* Framer (dsp/frame/framer.cc)                                             */
/* ======================================================================== */

struct or_framer {
    size_t n, h, c;
    int mode;
    float* buf;
    size_t cap, wpos, rpos;
};

/* Framer::reset (framer.cc:76-86) */
void or_framer_reset(or_framer* f) {
    free(f->buf);
    f->cap = f->n * f->c * 2;
    f->buf = (float*)calloc(f->cap ? f->cap : 1, sizeof(float));
    f->wpos = f->rpos = 0;
}

/* Framer::set_params (framer.cc:15-35) */
or_framer* or_framer_new(size_t n, size_t h, size_t c, int mode) {
    if (n == 0 || h == 0 || c == 0) return NULL;
    or_framer* f = (or_framer*)calloc(1, sizeof(or_framer));
    f->n = n;
    f->h = h;
    f->c = c;
    f->mode = mode;
    or_framer_reset(f);
    return f;
}

void or_framer_free(or_framer* f) {
    if (!f) return;
    free(f->buf);
    free(f);
}

/* Framer::resize_buffer_if_needed (framer.cc:120-126): doubling, zero fill */
static void framer_grow(or_framer* f, size_t need) {
    if (f->cap < need) {
        size_t nc = need > f->cap * 2 ? need : f->cap * 2;
        f->buf = (float*)realloc(f->buf, nc * sizeof(float));
        memset(f->buf + f->cap, 0, (nc - f->cap) * sizeof(float));
        f->cap = nc;
    }
}

/* Framer::push (framer.cc:37-59) */
int or_framer_push(or_framer* f, const float* x, size_t frames) {
    if (x == NULL && frames > 0) return 0;
    size_t add = frames * f->c;
    if (add == 0) return 1;
    framer_grow(f, f->wpos + add);
    memcpy(f->buf + f->wpos, x, add * sizeof(float));
    f->wpos += add;
    return 1;
}

/* Framer::calculate_available_frames (framer.cc:88-117) */
size_t or_framer_available(const or_framer* f) {
    if (f->wpos <= f->rpos) return 0;
    size_t avail = (f->wpos - f->rpos) / f->c;
    if (avail < f->n) {
        if (f->mode == OR_ZERO_PAD && avail > 0) return 1;
        return 0;
    }
    size_t nf = (avail - f->n) / f->h + 1;
    if (f->mode == OR_DROP) {
        size_t last = (nf - 1) * f->h;
        if (last + f->n > avail) nf = nf > 0 ? nf - 1 : 0;
    }
    return nf;
}

/* Framer::extract_frame (framer.cc:128-181) */
int or_framer_pop(or_framer* f, float* out) {
    if (out == NULL) return 0;
    if (or_framer_available(f) == 0) return 0;
    size_t start = f->rpos, fs = f->n * f->c;
    if (start + fs <= f->wpos) {
        memcpy(out, f->buf + start, fs * sizeof(float));
    } else {
        if (f->mode == OR_DROP) return 0;
        size_t av = f->wpos - start;
        if (av > 0) memcpy(out, f->buf + start, av * sizeof(float));
        for (size_t i = av; i < fs; ++i) out[i] = 0.0f;
    }
    f->rpos += f->h * f->c;
    if (f->rpos > f->wpos) f->rpos = f->wpos;
    if (f->rpos > f->cap / 2) { /* compaction (framer.cc:170-179) */
        size_t rem = f->rpos < f->wpos ? f->wpos - f->rpos : 0;
        if (rem > 0) memmove(f->buf, f->buf + f->rpos, rem * sizeof(float));
        f->wpos = rem;
        f->rpos = 0;
    }
    return 1;
}

/* ======================================================================== */
/* kissfft 131.1.0 restatement (float scalar, no fixed point)               */
/* ======================================================================== */

typedef struct { float r, i; } cpx;

#define MAXFACTORS 32
struct or_kfft_cfg {
    int nfft, inverse;
    int factors[2 * MAXFACTORS];
    cpx* twiddles;
    cpx* tmp; /* scratch for in-place calls and the generic butterfly */
};

/* C_MUL / C_ADD / C_SUB / C_ADDTO / HALF_OF from _kiss_fft_guts.h */
static inline cpx cmul(cpx a, cpx b) {
    cpx m;
    m.r = a.r * b.r - a.i * b.i;
    m.i = a.r * b.i + a.i * b.r;
    return m;
}
static inline cpx cadd(cpx a, cpx b) { cpx m = {a.r + b.r, a.i + b.i}; return m; }
static inline cpx csub(cpx a, cpx b) { cpx m = {a.r - b.r, a.i - b.i}; return m; }

/* kf_factor: powers of 4, then 2, then odd primes (kiss_fft.c) */
static void kf_factor(int n, int* facbuf) {
    int p = 4;
    double floor_sqrt = floor(sqrt((double)n));
    do {
        while (n % p) {
            switch (p) {
                case 4: p = 2; break;
                case 2: p = 3; break;
                default: p += 2; break;
            }
            if (p > floor_sqrt) p = n;
        }
        n /= p;
        *facbuf++ = p;
        *facbuf++ = n;
    } while (n > 1);
}

or_kfft_cfg* or_kfft_alloc(int nfft, int inverse) {
    if (nfft <= 0) return NULL;
    or_kfft_cfg* st = (or_kfft_cfg*)calloc(1, sizeof(or_kfft_cfg));
    st->nfft = nfft;
    st->inverse = inverse;
    st->twiddles = (cpx*)malloc(sizeof(cpx) * (size_t)nfft);
    st->tmp = (cpx*)malloc(sizeof(cpx) * (size_t)nfft);
    for (int i = 0; i < nfft; ++i) {
        const double pi = 3.141592653589793238462643383279502884197169399375105820974944;
        double phase = -2 * pi * i / nfft;
        if (inverse) phase *= -1;
        st->twiddles[i].r = (float)cos(phase); /* kf_cexp */
        st->twiddles[i].i = (float)sin(phase);
    }
    kf_factor(nfft, st->factors);
    return st;
}

void or_kfft_free(or_kfft_cfg* st) {
    if (!st) return;
    free(st->twiddles);
    free(st->tmp);
    free(st);
}

static void kf_bfly2(cpx* Fout, size_t fstride, const or_kfft_cfg* st, int m) {
    cpx* Fout2 = Fout + m;
    const cpx* tw1 = st->twiddles;
    do {
        cpx t = cmul(*Fout2, *tw1);
        tw1 += fstride;
        *Fout2 = csub(*Fout, t);
        *Fout = cadd(*Fout, t);
        ++Fout2;
        ++Fout;
    } while (--m);
}

static void kf_bfly4(cpx* Fout, size_t fstride, const or_kfft_cfg* st, size_t m) {
    const cpx *tw1, *tw2, *tw3;
    cpx s[6];
    size_t k = m;
    const size_t m2 = 2 * m, m3 = 3 * m;
    tw3 = tw2 = tw1 = st->twiddles;
    do {
        s[0] = cmul(Fout[m], *tw1);
        s[1] = cmul(Fout[m2], *tw2);
        s[2] = cmul(Fout[m3], *tw3);
        s[5] = csub(*Fout, s[1]);
        *Fout = cadd(*Fout, s[1]);
        s[3] = cadd(s[0], s[2]);
        s[4] = csub(s[0], s[2]);
        Fout[m2] = csub(*Fout, s[3]);
        tw1 += fstride;
        tw2 += fstride * 2;
        tw3 += fstride * 3;
        *Fout = cadd(*Fout, s[3]);
        if (st->inverse) {
            Fout[m].r = s[5].r - s[4].i;
            Fout[m].i = s[5].i + s[4].r;
            Fout[m3].r = s[5].r + s[4].i;
            Fout[m3].i = s[5].i - s[4].r;
        } else {
            Fout[m].r = s[5].r + s[4].i;
            Fout[m].i = s[5].i - s[4].r;
            Fout[m3].r = s[5].r - s[4].i;
            Fout[m3].i = s[5].i + s[4].r;
        }
        ++Fout;
    } while (--k);
}

static void kf_bfly3(cpx* Fout, size_t fstride, const or_kfft_cfg* st, size_t m) {
    size_t k = m;
    const size_t m2 = 2 * m;
    const cpx *tw1, *tw2;
    cpx s[5];
    cpx epi3 = st->twiddles[fstride * m];
    tw1 = tw2 = st->twiddles;
    do {
        s[1] = cmul(Fout[m], *tw1);
        s[2] = cmul(Fout[m2], *tw2);
        s[3] = cadd(s[1], s[2]);
        s[0] = csub(s[1], s[2]);
        tw1 += fstride;
        tw2 += fstride * 2;
        Fout[m].r = Fout->r - s[3].r * 0.5f;
        Fout[m].i = Fout->i - s[3].i * 0.5f;
        s[0].r *= epi3.i;
        s[0].i *= epi3.i;
        *Fout = cadd(*Fout, s[3]);
        Fout[m2].r = Fout[m].r + s[0].i;
        Fout[m2].i = Fout[m].i - s[0].r;
        Fout[m].r -= s[0].i;
        Fout[m].i += s[0].r;
        ++Fout;
    } while (--k);
}

static void kf_bfly5(cpx* Fout, size_t fstride, const or_kfft_cfg* st, int m) {
    cpx *F0, *F1, *F2, *F3, *F4;
    cpx s[13];
    const cpx* tw = st->twiddles;
    cpx ya = tw[fstride * m];
    cpx yb = tw[fstride * 2 * m];
    F0 = Fout;
    F1 = F0 + m;
    F2 = F0 + 2 * m;
    F3 = F0 + 3 * m;
    F4 = F0 + 4 * m;
    for (int u = 0; u < m; ++u) {
        s[0] = *F0;
        s[1] = cmul(*F1, tw[u * fstride]);
        s[2] = cmul(*F2, tw[2 * u * fstride]);
        s[3] = cmul(*F3, tw[3 * u * fstride]);
        s[4] = cmul(*F4, tw[4 * u * fstride]);
        s[7] = cadd(s[1], s[4]);
        s[10] = csub(s[1], s[4]);
        s[8] = cadd(s[2], s[3]);
        s[9] = csub(s[2], s[3]);
        F0->r += s[7].r + s[8].r;
        F0->i += s[7].i + s[8].i;
        s[5].r = s[0].r + s[7].r * ya.r + s[8].r * yb.r;
        s[5].i = s[0].i + s[7].i * ya.r + s[8].i * yb.r;
        s[6].r = s[10].i * ya.i + s[9].i * yb.i;
        s[6].i = -(s[10].r * ya.i) - s[9].r * yb.i;
        *F1 = csub(s[5], s[6]);
        *F4 = cadd(s[5], s[6]);
        s[11].r = s[0].r + s[7].r * yb.r + s[8].r * ya.r;
        s[11].i = s[0].i + s[7].i * yb.r + s[8].i * ya.r;
        s[12].r = -(s[10].i * yb.i) + s[9].i * ya.i;
        s[12].i = s[10].r * yb.i - s[9].r * ya.i;
        *F2 = cadd(s[11], s[12]);
        *F3 = csub(s[11], s[12]);
        ++F0; ++F1; ++F2; ++F3; ++F4;
    }
}

static void kf_bfly_generic(cpx* Fout, size_t fstride, const or_kfft_cfg* st, int m, int p) {
    const cpx* tw = st->twiddles;
    int norig = st->nfft;
    cpx* scratch = (cpx*)malloc(sizeof(cpx) * (size_t)p);
    for (int u = 0; u < m; ++u) {
        int k = u;
        for (int q1 = 0; q1 < p; ++q1) {
            scratch[q1] = Fout[k];
            k += m;
        }
        k = u;
        for (int q1 = 0; q1 < p; ++q1) {
            int twidx = 0;
            Fout[k] = scratch[0];
            for (int q = 1; q < p; ++q) {
                twidx += (int)fstride * k;
                if (twidx >= norig) twidx -= norig;
                cpx t = cmul(scratch[q], tw[twidx]);
                Fout[k] = cadd(Fout[k], t);
            }
            k += m;
        }
    }
    free(scratch);
}

/* kf_work: recursive decimation in time (kiss_fft.c) */
static void kf_work(cpx* Fout, const cpx* f, size_t fstride, int in_stride, const int* factors,
                    const or_kfft_cfg* st) {
    cpx* Fout_beg = Fout;
    const int p = *factors++;
    const int m = *factors++;
    const cpx* Fout_end = Fout + p * m;
    if (m == 1) {
        do {
            *Fout = *f;
            f += fstride * (size_t)in_stride;
        } while (++Fout != Fout_end);
    } else {
        do {
            kf_work(Fout, f, fstride * (size_t)p, in_stride, factors, st);
            f += fstride * (size_t)in_stride;
        } while ((Fout += m) != Fout_end);
    }
    Fout = Fout_beg;
    switch (p) {
        case 2: kf_bfly2(Fout, fstride, st, m); break;
        case 3: kf_bfly3(Fout, fstride, st, (size_t)m); break;
        case 4: kf_bfly4(Fout, fstride, st, (size_t)m); break;
        case 5: kf_bfly5(Fout, fstride, st, m); break;
        default: kf_bfly_generic(Fout, fstride, st, m, p); break;
    }
}

/* kiss_fft / kiss_fft_stride: in-place goes through a temp buffer */
void or_kfft(or_kfft_cfg* st, const float* fin, float* fout) {
    const cpx* in = (const cpx*)fin;
    cpx* out = (cpx*)fout;
    if (in == out) {
        kf_work(st->tmp, in, 1, 1, st->factors, st);
        memcpy(out, st->tmp, sizeof(cpx) * (size_t)st->nfft);
    } else {
        kf_work(out, in, 1, 1, st->factors, st);
    }
}

struct or_kfftr_cfg {
    or_kfft_cfg* sub;
    cpx* tmpbuf;
    cpx* super_twiddles;
};

/* kiss_fftr_alloc: half-size complex plan + super twiddles */
or_kfftr_cfg* or_kfftr_alloc(int nfft, int inverse) {
    if (nfft <= 0 || (nfft & 1)) return NULL;
    or_kfftr_cfg* st = (or_kfftr_cfg*)calloc(1, sizeof(or_kfftr_cfg));
    int ncfft = nfft >> 1;
    st->sub = or_kfft_alloc(ncfft, inverse);
    st->tmpbuf = (cpx*)malloc(sizeof(cpx) * (size_t)ncfft);
    st->super_twiddles = (cpx*)malloc(sizeof(cpx) * (size_t)(ncfft / 2 + 1));
    for (int i = 0; i < ncfft / 2; ++i) {
        double phase = -3.14159265358979323846264338327 * ((double)(i + 1) / ncfft + .5);
        if (inverse) phase *= -1;
        st->super_twiddles[i].r = (float)cos(phase);
        st->super_twiddles[i].i = (float)sin(phase);
    }
    return st;
}

void or_kfftr_free(or_kfftr_cfg* st) {
    if (!st) return;
    or_kfft_free(st->sub);
    free(st->tmpbuf);
    free(st->super_twiddles);
    free(st);
}

/* kiss_fftr */
void or_kfftr(or_kfftr_cfg* st, const float* timedata, float* freqdata_f) {
    cpx* freq = (cpx*)freqdata_f;
    int ncfft = st->sub->nfft;
    kf_work(st->tmpbuf, (const cpx*)timedata, 1, 1, st->sub->factors, st->sub);
    cpx tdc = st->tmpbuf[0];
    freq[0].r = tdc.r + tdc.i;
    freq[ncfft].r = tdc.r - tdc.i;
    freq[ncfft].i = freq[0].i = 0;
    for (int k = 1; k <= ncfft / 2; ++k) {
        cpx fpk = st->tmpbuf[k];
        cpx fpnk;
        fpnk.r = st->tmpbuf[ncfft - k].r;
        fpnk.i = -st->tmpbuf[ncfft - k].i;
        cpx f1k = cadd(fpk, fpnk);
        cpx f2k = csub(fpk, fpnk);
        cpx tw = cmul(f2k, st->super_twiddles[k - 1]);
        freq[k].r = (f1k.r + tw.r) * 0.5f;
        freq[k].i = (f1k.i + tw.i) * 0.5f;
        freq[ncfft - k].r = (f1k.r - tw.r) * 0.5f;
        freq[ncfft - k].i = (tw.i - f1k.i) * 0.5f;
    }
}

/* kiss_fftri */
void or_kfftri(or_kfftr_cfg* st, const float* freqdata_f, float* timedata) {
    const cpx* freq = (const cpx*)freqdata_f;
    int ncfft = st->sub->nfft;
    st->tmpbuf[0].r = freq[0].r + freq[ncfft].r;
    st->tmpbuf[0].i = freq[0].r - freq[ncfft].r;
    for (int k = 1; k <= ncfft / 2; ++k) {
        cpx fk = freq[k];
        cpx fnkc;
        fnkc.r = freq[ncfft - k].r;
        fnkc.i = -freq[ncfft - k].i;
        cpx fek = cadd(fk, fnkc);
        cpx tmp = csub(fk, fnkc);
        cpx fok = cmul(tmp, st->super_twiddles[k - 1]);
        st->tmpbuf[k] = cadd(fek, fok);
        st->tmpbuf[ncfft - k] = csub(fek, fok);
        st->tmpbuf[ncfft - k].i *= -1;
    }
    kf_work((cpx*)timedata, st->tmpbuf, 1, 1, st->sub->factors, st->sub);
}

/* ======================================================================== */
/* KissFftPlan adapter semantics (dsp/fft/backends/kissfft_adapter.cc)      */
/* ======================================================================== */

/* sanitize: NaN/Inf -> 0, |v| < 1e-30 -> 0 (kissfft_adapter.cc:102-110, 156-163) */
static inline float sanit(float v) {
    if (isnan(v) || isinf(v)) return 0.0f;
    if (fabsf(v) < 1e-30f) return 0.0f;
    return v;
}

void or_adapter_forward(or_kfftr_cfg* fwd, int nfft, const float* in, float* out) {
    float* clean = (float*)malloc(sizeof(float) * (size_t)nfft);
    for (int i = 0; i < nfft; ++i) clean[i] = sanit(in[i]);
    or_kfftr(fwd, clean, out);
    free(clean);
}

void or_adapter_inverse(or_kfftr_cfg* inv, int nfft, const float* in, float* out) {
    float* tmp = (float*)malloc(sizeof(float) * (size_t)nfft);
    or_kfftri(inv, in, tmp);
    const float scale = 1.0f / (float)nfft; /* :154 */
    for (int i = 0; i < nfft; ++i) out[i] = sanit(tmp[i] * scale);
    free(tmp);
}

/* kissfft_adapter.cc:171-202: no sanitize on the forward complex path */
void or_adapter_forward_complex(or_kfft_cfg* fwd, int nfft, const float* in, float* out) {
    float* buf = (float*)malloc(sizeof(float) * 2 * (size_t)nfft);
    memcpy(buf, in, sizeof(float) * 2 * (size_t)nfft);
    or_kfft(fwd, buf, buf);
    memcpy(out, buf, sizeof(float) * 2 * (size_t)nfft);
    free(buf);
}

/* kissfft_adapter.cc:204-246 */
void or_adapter_inverse_complex(or_kfft_cfg* inv, int nfft, const float* in, float* out) {
    float* buf = (float*)malloc(sizeof(float) * 2 * (size_t)nfft);
    memcpy(buf, in, sizeof(float) * 2 * (size_t)nfft);
    or_kfft(inv, buf, buf);
    const float scale = 1.0f / (float)nfft;
    for (int i = 0; i < nfft; ++i) {
        float re = buf[2 * i] * scale, im = buf[2 * i + 1] * scale;
        if (isnan(re) || isinf(re) || fabsf(re) < 1e-30f) re = 0.0f;
        if (isnan(im) || isinf(im) || fabsf(im) < 1e-30f) im = 0.0f;
        out[2 * i] = re;
        out[2 * i + 1] = im;
    }
    free(buf);
}

/* ======================================================================== */
/* OLA kernels, scalar references (dsp/ola/kernels.cc:18-36)                */
/* ======================================================================== */

void or_axpy(float* dst, const float* src, float g, size_t n) {
    for (size_t i = 0; i < n; ++i) dst[i] = fmaf(src[i], g, dst[i]);
}

void or_axpy_windowed(float* dst, const float* src, const float* win, float g, size_t n) {
    for (size_t i = 0; i < n; ++i) dst[i] = fmaf(fmaf(src[i], win[i], 0.0f), g, dst[i]);
}

void or_normalize_and_clear(float* out, float* acc, const float* norm, float eps, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const float d = (norm[i] > eps) ? norm[i] : eps;
        out[i] = acc[i] / d;
        acc[i] = 0.0f;
    }
}

/* ======================================================================== */
/* OLAAccumulator (dsp/ola/OLAAccumulator.cc)                               */
/* ======================================================================== */

struct or_ola {
    size_t n, h, c, ring_len;
    float eps;
    int inside;
    float* window; /* NULL until set_window */
    float* ring;   /* c * ring_len */
    float* norm;
    float* scratch;
    size_t read_pos, produced;
    float meter_peak;
};

or_ola* or_ola_new(size_t n, size_t h, size_t c, float eps, int inside) {
    if (n == 0 || h == 0 || c == 0 || !(eps > 0.0f)) return NULL; /* OLAConfig::isValid */
    or_ola* o = (or_ola*)calloc(1, sizeof(or_ola));
    o->n = n;
    o->h = h;
    o->c = c;
    o->eps = eps;
    o->inside = inside;
    o->ring_len = or_ring_len(n, h);
    o->ring = (float*)calloc(c * o->ring_len, sizeof(float));
    o->norm = (float*)malloc(sizeof(float) * o->ring_len);
    o->scratch = (float*)malloc(sizeof(float) * c * n);
    or_init_normalization(o->norm, NULL, o->ring_len, n, h, inside, eps);
    return o;
}

void or_ola_free(or_ola* o) {
    if (!o) return;
    free(o->window);
    free(o->ring);
    free(o->norm);
    free(o->scratch);
    free(o);
}

/* OLAAccumulator::set_window (OLAAccumulator.cc:38-52) */
void or_ola_set_window(or_ola* o, const float* w) {
    if (!o->window) o->window = (float*)malloc(sizeof(float) * o->n);
    memcpy(o->window, w, sizeof(float) * o->n);
    or_init_normalization(o->norm, o->window, o->ring_len, o->n, o->h, o->inside, o->eps);
}

/* RingBuffer::split (ring_buffer.cc:44-85): len clamped to capacity */
static void ring_split(size_t cap, size_t start, size_t len, size_t* s1, size_t* l1,
                       size_t* l2) {
    if (len > cap) len = cap;
    start %= cap;
    if (start + len <= cap) {
        *s1 = start;
        *l1 = len;
        *l2 = 0;
    } else {
        *s1 = start;
        *l1 = cap - start;
        *l2 = len - *l1;
    }
}

/* exported for the pins against the reference's compiled ring_buffer.cc */
void or_ring_split(size_t cap, size_t start, size_t len, size_t* s1, size_t* l1, size_t* l2) {
    ring_split(cap, start, len, s1, l1, l2);
}

/* ola::deinterleave_to_scratch (aos_to_soa.cc:7-18): [i][ch] -> [ch][i] */
void or_deinterleave(const float* x, size_t n, size_t channels, float* scratch) {
    if (!x || !scratch || n == 0 || channels == 0) return;
    for (size_t ch = 0; ch < channels; ++ch)
        for (size_t i = 0; i < n; ++i) scratch[ch * n + i] = x[i * channels + ch];
}

/* OLAAccumulator::add_frame_SoA (OLAAccumulator.cc:54-122) */
void or_ola_add_frame_soa(or_ola* o, const float* const* ch, const float* window,
                          size_t start_sample, size_t start_off, size_t size, float gain) {
    if (size == 0) return;
    if (start_off >= o->n) return;
    size_t eff = size;
    if (start_off + size > o->n) eff = o->n - start_off;
    for (size_t c = 0; c < o->c; ++c) {
        int use_win = o->inside ? (o->window != NULL) : (window != NULL);
        const float* w = use_win ? (o->inside ? o->window : window) : NULL;
        float* ring = o->ring + c * o->ring_len;
        size_t s1, l1, l2;
        ring_split(o->ring_len, start_sample, eff, &s1, &l1, &l2);
        if (l1) {
            if (use_win)
                or_axpy_windowed(ring + s1, ch[c] + start_off, w + start_off, gain, l1);
            else
                or_axpy(ring + s1, ch[c] + start_off, gain, l1);
        }
        if (l2) {
            if (use_win)
                or_axpy_windowed(ring, ch[c] + start_off + l1, w + start_off + l1, gain, l2);
            else
                or_axpy(ring, ch[c] + start_off + l1, gain, l2);
        }
    }
    if (start_sample + eff > o->produced) o->produced = start_sample + eff;
}

/* OLAAccumulator::push_frame_AoS (OLAAccumulator.cc:124-160), aos_to_soa.cc:7-18 */
void or_ola_push_frame_aos(or_ola* o, const float* x, const float* window, size_t start_sample,
                           size_t start_off, size_t size, float gain) {
    if (size == 0) return;
    if (start_off >= o->n) return;
    size_t eff = size;
    if (start_off + size > o->n) eff = o->n - start_off;
    or_deinterleave(x + start_off * o->c, eff, o->c, o->scratch);
    const float* ptrs[64] = {0};
    const float** chp = o->c <= 64 ? ptrs : (const float**)malloc(sizeof(float*) * o->c);
    for (size_t ch = 0; ch < o->c; ++ch) chp[ch] = o->scratch + ch * eff;
    or_ola_add_frame_soa(o, chp, window, start_sample, 0, eff, gain);
    if (chp != ptrs) free((void*)chp);
}

/* OLAAccumulator::produce (OLAAccumulator.cc:162-221) */
size_t or_ola_produce(or_ola* o, float* const* out, size_t n) {
    if (n == 0) return 0;
    size_t avail = o->produced > o->read_pos ? o->produced - o->read_pos : 0;
    if (avail == 0) return 0;
    if (avail < n) n = avail;
    for (size_t c = 0; c < o->c; ++c) {
        float* ring = o->ring + c * o->ring_len;
        size_t s1, l1, l2;
        ring_split(o->ring_len, o->read_pos, n, &s1, &l1, &l2);
        if (l1) or_normalize_and_clear(out[c], ring + s1, o->norm + s1, o->eps, l1);
        if (l2) or_normalize_and_clear(out[c] + l1, ring, o->norm, o->eps, l2);
    }
    o->read_pos = (o->read_pos + n) % o->ring_len; /* :213 */
    for (size_t i = 0; i < n; ++i) {                /* update_peak_meter :290-295 */
        float a = fabsf(out[0][i]);
        if (a > o->meter_peak) o->meter_peak = a;
    }
    return n;
}

/* OLAAccumulator::flush (OLAAccumulator.cc:223-228): counters only */
void or_ola_flush(or_ola* o) {
    if (o->read_pos + o->n > o->produced) o->produced = o->read_pos + o->n;
}

/* OLAAccumulator::reset (OLAAccumulator.cc:230-247): rings zeroed, window dropped */
void or_ola_reset(or_ola* o) {
    memset(o->ring, 0, sizeof(float) * o->c * o->ring_len);
    o->read_pos = 0;
    o->produced = 0;
    o->meter_peak = 0.0f;
    free(o->window);
    o->window = NULL;
    or_init_normalization(o->norm, NULL, o->ring_len, o->n, o->h, o->inside, o->eps);
}

size_t or_ola_ring_size(const or_ola* o) { return o->ring_len; }
const float* or_ola_norm(const or_ola* o) { return o->norm; }
size_t or_ola_produced(const or_ola* o) { return o->produced; }
size_t or_ola_read_pos(const or_ola* o) { return o->read_pos; }
float or_ola_meter_peak(const or_ola* o) { return o->meter_peak; }

/* ======================================================================== */
/* The round trip (bench/e2e_benchmark.cc:138-186, streaming-interleaved)   */
/* ======================================================================== */

size_t or_frame_count(size_t T, size_t n, size_t h, int mode) {
    if (T == 0) return 0;
    if (mode == OR_ZERO_PAD) return (T + h - 1) / h;
    if (T < n) return 0;
    return (T - n) / h + 1;
}

/* ======================================================================== */
/* FrameQueue (dsp/frame/FrameQueue.cc, dsp/frame/Indexing.h)               */
/* ======================================================================== */

/* Indexing.h:18-37: left side i -> -i-1 (-1 -> 0), right side i -> 2n-2-i
 * (n -> n-2), repeated until inside. */
int or_fq_reflect101(int i, int n) {
    if (n <= 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0)
            i = -i - 1;
        else
            i = 2 * n - 2 - i;
    }
    return i;
}

/* Indexing.h:48-68 getPaddingValueSafe */
float or_fq_pad_value(const float* data, int len, int idx, int pad_mode) {
    if (len <= 0) return 0.0f;
    switch (pad_mode) {
        case 0: return 0.0f;
        case 2: return idx < 0 ? data[0] : idx >= len ? data[len - 1] : data[idx];
        case 1: return data[or_fq_reflect101(idx, len)];
        default: return 0.0f;
    }
}

/* FrameQueue.cc:98-115 calculateNumFrames on the padded length */
size_t or_fq_count(size_t T, size_t n, size_t h, int center) {
    const size_t padded = T + (center ? 2 * (n / 2) : 0);
    if (padded < n) return 0;
    const size_t tail = n > h ? n - h : 0;
    if (padded < tail) return 0;
    return (padded - tail) / h;
}

/* FrameQueue.cc:9-45 + createPaddedInput (:66-96) */
size_t or_fq_frames(const float* x, size_t T, size_t n, size_t h, int center, int pad_mode,
                    float* frames) {
    const size_t pad = center ? n / 2 : 0;
    const size_t padded_len = T + 2 * pad;
    float* padded = (float*)malloc(sizeof(float) * (padded_len ? padded_len : 1));
    if (!center) {
        if (T) memcpy(padded, x, sizeof(float) * T);
    } else {
        const int sl = (int)T, sp = (int)pad;
        for (int i = -sp; i < sl + sp; ++i)
            padded[i + sp] = (i >= 0 && i < sl) ? x[i] : or_fq_pad_value(x, sl, i, pad_mode);
    }
    const size_t F = or_fq_count(T, n, h, center);
    if (frames) {
        for (size_t k = 0; k < F; ++k)
            for (size_t i = 0; i < n; ++i) {
                const size_t idx = k * h + i;
                frames[k * n + i] = idx < padded_len
                                        ? padded[idx]
                                        : or_fq_pad_value(padded, (int)padded_len, (int)idx, pad_mode);
            }
    }
    free(padded);
    return F;
}

long or_roundtrip(const float* x, size_t T, size_t n, size_t h, int wtype, int periodic, int mode,
                  float* y, size_t y_cap, float* frames_out, float* spec_out) {
    return or_roundtrip_ex(x, T, n, h, wtype, periodic, mode, 0, 0, 1, y, y_cap, frames_out,
                           spec_out);
}

static long or_roundtrip_impl(const float* x, size_t T, size_t n, size_t h, int wtype, int periodic,
                              int framing, int center, int pad_mode, int analysis_window, const float* bin_gain,
                              const float* mask, size_t mask_ld, float* y, size_t y_cap, float* frames_out,
                              float* spec_out, float* raw_spec_out);

long or_roundtrip_ex(const float* x, size_t T, size_t n, size_t h, int wtype, int periodic,
                     int framing, int center, int pad_mode, int analysis_window, float* y,
                     size_t y_cap, float* frames_out, float* spec_out) {
    return or_roundtrip_impl(x, T, n, h, wtype, periodic, framing, center, pad_mode, analysis_window, NULL, NULL, 0,
                             y, y_cap, frames_out, spec_out, NULL);
}

/* The same loop with a spectral step where e2e_benchmark.cc:161-162 puts one
 * ("filtering or other processing could go here"): every bin of each frame's
 * spectrum scaled by bin_gain[k] (n/2+1 real gains; re and im multiplied, as a
 * caller editing the interleaved complex spectrum on the host would). */
long or_roundtrip_gain(const float* x, size_t T, size_t n, size_t h, int wtype, int periodic, int framing,
                       const float* bin_gain, float* y, size_t y_cap) {
    return or_roundtrip_impl(x, T, n, h, wtype, periodic, framing, 0, 0, 1, bin_gain, NULL, 0, y, y_cap, NULL, NULL,
                             NULL);
}

/* The same loop with a time-varying spectral step (crlot_plan_set_spectral_mask):
 * frame k's spectrum is scaled by bin_gain[b] (nullable), then by mask row k,
 * mask[k * mask_ld + b] (nullable), b <= n/2 -- re and im each multiplied, as in
 * or_roundtrip_gain.  raw_spec_out (nullable, rows of n + 2 floats) receives the
 * forward spectra before the step: IFftPlan::forward of frame * w, what
 * crlot_stft writes. */
long or_roundtrip_mask(const float* x, size_t T, size_t n, size_t h, int wtype, int periodic, int framing,
                       int center, int pad_mode, int analysis_window, const float* bin_gain, const float* mask,
                       size_t mask_ld, float* y, size_t y_cap, float* raw_spec_out) {
    return or_roundtrip_impl(x, T, n, h, wtype, periodic, framing, center, pad_mode, analysis_window, bin_gain,
                             mask, mask_ld, y, y_cap, NULL, NULL, raw_spec_out);
}

static long or_roundtrip_impl(const float* x, size_t T, size_t n, size_t h, int wtype, int periodic,
                              int framing, int center, int pad_mode, int analysis_window, const float* bin_gain,
                              const float* mask, size_t mask_ld, float* y, size_t y_cap, float* frames_out,
                              float* spec_out, float* raw_spec_out) {
    if (n == 0 || h == 0 || (n & 1)) return -1;
    if (framing < 0 || framing > 2) return -3;
    float* w = (float*)malloc(sizeof(float) * n);
    if (or_window(wtype, n, periodic, OR_NORM_NONE, w) != 0) {
        free(w);
        return -2;
    }
    or_framer* fr = NULL;
    float* fq = NULL;
    size_t fq_n = 0;
    if (framing == 2) {
        fq_n = or_fq_count(T, n, h, center);
        fq = (float*)malloc(sizeof(float) * (fq_n * n + 1));
        or_fq_frames(x, T, n, h, center, pad_mode, fq);
    } else {
        fr = or_framer_new(n, h, 1, framing);
        or_framer_push(fr, x, T);
    }
    or_ola* ola = or_ola_new(n, h, 1, 1e-8f, 1);
    or_ola_set_window(ola, w);
    or_kfftr_cfg* fwd = or_kfftr_alloc((int)n, 0);
    or_kfftr_cfg* inv = or_kfftr_alloc((int)n, 1);
    float* frame = (float*)malloc(sizeof(float) * n);
    float* proc = (float*)malloc(sizeof(float) * n);
    float* spec = (float*)malloc(sizeof(float) * (n + 2));
    float* tmp = (float*)malloc(sizeof(float) * h);
    size_t k = 0, out_pos = 0;
    for (;;) {
        if (fr) {
            if (!or_framer_pop(fr, frame)) break;
        } else {
            if (k >= fq_n) break;
            memcpy(frame, fq + k * n, sizeof(float) * n); /* FrameQueue::getFrame */
        }
        for (size_t i = 0; i < n; ++i) /* e2e_benchmark.cc:154-156 (analysis window) */
            proc[i] = analysis_window ? frame[i] * w[i] : frame[i];
        or_adapter_forward(fwd, (int)n, proc, spec);
        if (raw_spec_out) memcpy(raw_spec_out + k * (n + 2), spec, sizeof(float) * (n + 2));
        if (bin_gain)
            for (size_t b = 0; b <= n / 2; ++b) {
                spec[2 * b] *= bin_gain[b];
                spec[2 * b + 1] *= bin_gain[b];
            }
        if (mask)
            for (size_t b = 0; b <= n / 2; ++b) {
                spec[2 * b] *= mask[k * mask_ld + b];
                spec[2 * b + 1] *= mask[k * mask_ld + b];
            }
        if (spec_out) memcpy(spec_out + k * (n + 2), spec, sizeof(float) * (n + 2));
        or_adapter_inverse(inv, (int)n, spec, proc);
        if (frames_out) memcpy(frames_out + k * n, proc, sizeof(float) * n);
        or_ola_push_frame_aos(ola, proc, NULL, k * h, 0, n, 1.0f);
        float* chp[1] = {tmp};
        const size_t got = or_ola_produce(ola, chp, h);
        if (out_pos < y_cap) {
            const size_t cp = y_cap - out_pos < got ? y_cap - out_pos : got;
            memcpy(y + out_pos, tmp, sizeof(float) * cp);
        }
        out_pos += got;
        ++k;
    }
    free(frame);
    free(proc);
    free(spec);
    free(tmp);
    free(w);
    free(fq);
    or_kfftr_free(fwd);
    or_kfftr_free(inv);
    or_ola_free(ola);
    if (fr) or_framer_free(fr);
    return (long)k;
}

/* bench/e2e_benchmark.cc:152-179 in its literal order: every frame pushed
 * (pop -> window -> forward -> inverse -> push_frame_AoS(k H)), THEN the produce
 * loop asking for what is left of T each call -- the ring aliases when the
 * signal outruns the ring, as the reference's does.  Returns the
 * samples produced (at most y_cap are stored). */
long or_roundtrip_harness_order(const float* x, size_t T, size_t n, size_t h, int wtype, int periodic, float* y,
                                size_t y_cap) {
    if (n == 0 || h == 0 || (n & 1)) return -1;
    float* w = (float*)malloc(sizeof(float) * n);
    if (or_window(wtype, n, periodic, OR_NORM_NONE, w) != 0) {
        free(w);
        return -2;
    }
    or_framer* fr = or_framer_new(n, h, 1, OR_ZERO_PAD);
    or_framer_push(fr, x, T);
    or_ola* ola = or_ola_new(n, h, 1, 1e-8f, 1);
    or_ola_set_window(ola, w);
    or_kfftr_cfg* fwd = or_kfftr_alloc((int)n, 0);
    or_kfftr_cfg* inv = or_kfftr_alloc((int)n, 1);
    float* frame = (float*)malloc(sizeof(float) * n);
    float* proc = (float*)malloc(sizeof(float) * n);
    float* spec = (float*)malloc(sizeof(float) * (n + 2));
    size_t k = 0;
    while (or_framer_pop(fr, frame)) {
        for (size_t i = 0; i < n; ++i) proc[i] = frame[i] * w[i];
        or_adapter_forward(fwd, (int)n, proc, spec);
        or_adapter_inverse(inv, (int)n, spec, proc);
        or_ola_push_frame_aos(ola, proc, NULL, k * h, 0, n, 1.0f);
        ++k;
    }
    size_t got = 0;
    float* tmp = (float*)calloc(T + 1, sizeof(float)); /* (a clamped read leaves its tail as it was) */
    while (got < T) {
        float* chp[1] = {tmp};
        const size_t s = or_ola_produce(ola, chp, T - got);
        if (s == 0) break;
        if (got < y_cap) memcpy(y + got, tmp, sizeof(float) * (y_cap - got < s ? y_cap - got : s));
        got += s;
    }
    free(tmp);
    free(frame);
    free(proc);
    free(spec);
    free(w);
    or_kfftr_free(fwd);
    or_kfftr_free(inv);
    or_ola_free(ola);
    or_framer_free(fr);
    return (long)got;
}

typedef struct {
    const float* x;
    float* y;
    size_t s0, s1, T, ld_x, ld_y, n, h;
    int wtype, periodic, mode, center, pad_mode, analysis_window;
    long ret;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    j->ret = 0;
    for (size_t s = j->s0; s < j->s1; ++s) {
        long r = or_roundtrip_ex(j->x + s * j->ld_x, j->T, j->n, j->h, j->wtype, j->periodic,
                                 j->mode, j->center, j->pad_mode, j->analysis_window,
                                 j->y + s * j->ld_y, j->ld_y, NULL, NULL);
        if (r < 0) {
            j->ret = r;
            break;
        }
        j->ret = r;
    }
    return NULL;
}

long or_roundtrip_batch(const float* x, size_t n_streams, size_t T, size_t ld_x, size_t n,
                        size_t h, int wtype, int periodic, int mode, float* y, size_t ld_y,
                        int nthreads) {
    return or_roundtrip_batch_ex(x, n_streams, T, ld_x, n, h, wtype, periodic, mode, 0, 0, 1, y,
                                 ld_y, nthreads);
}

long or_roundtrip_batch_ex(const float* x, size_t n_streams, size_t T, size_t ld_x, size_t n,
                           size_t h, int wtype, int periodic, int mode, int center, int pad_mode,
                           int analysis_window, float* y, size_t ld_y, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n_streams) nthreads = (int)(n_streams ? n_streams : 1);
    batch_job* jobs = (batch_job*)calloc((size_t)nthreads, sizeof(batch_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        batch_job* j = &jobs[t];
        j->x = x;
        j->y = y;
        j->s0 = n_streams * (size_t)t / (size_t)nthreads;
        j->s1 = n_streams * (size_t)(t + 1) / (size_t)nthreads;
        j->T = T;
        j->ld_x = ld_x;
        j->ld_y = ld_y;
        j->n = n;
        j->h = h;
        j->wtype = wtype;
        j->periodic = periodic;
        j->mode = mode;
        j->center = center;
        j->pad_mode = pad_mode;
        j->analysis_window = analysis_window;
        pthread_create(&th[t], NULL, batch_worker, j);
    }
    long ret = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].ret < 0) ret = jobs[t].ret;
        else if (ret >= 0) ret = jobs[t].ret;
    }
    free(jobs);
    free(th);
    return ret;
}

/* splitmix64 -> uniform float in [-1, 1) * 0.5 (SURVEY.md 8d synthetic inputs) */
void or_synth_fill(float* x, size_t n, unsigned long long seed) {
    uint64_t s = seed;
    for (size_t i = 0; i < n; ++i) {
        uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z = z ^ (z >> 31);
        /* top 24 bits -> [0,1) exactly representable, then [-1,1), then *0.5 */
        float u = (float)(z >> 40) * (1.0f / 16777216.0f);
        x[i] = (u * 2.0f - 1.0f) * 0.5f;
    }
}

/* ---- bench.py cpu_baseline helpers: the reference harnesses' per-frame call
 * sequences run in C (no Python per call).  Test/measurement infrastructure. */

/* ola_benchmark.cc ParamAddFrameSoA + ParamProduce in streaming order over F
 * frames of c channels: add_frame_SoA(frame k, window, k*h, 0, n, gain) then
 * produce(h).  frames: [F][c][n]; out: [c][F*h]. */
void or_bench_ola_stream(size_t n, size_t h, size_t c, int inside, const float* window,
                         const float* frames, int64_t F, float gain, float* out) {
    or_ola* o = or_ola_new(n, h, c, 1e-8f, inside);
    if (!o) return;
    or_ola_set_window(o, window);
    const float* ch[64];
    float* och[64];
    for (int64_t k = 0; k < F; ++k) {
        for (size_t j = 0; j < c && j < 64; ++j) {
            ch[j] = frames + ((size_t)k * c + j) * n;
            och[j] = out + j * (size_t)F * h + (size_t)k * h;
        }
        or_ola_add_frame_soa(o, ch, window, (size_t)k * h, 0, n, gain);
        or_ola_produce(o, och, h);
    }
    or_ola_free(o);
}

/* micro_fft_benchmark.cc: IFftPlan::forward over B frames of nfft samples. */
void or_bench_rfft(int nfft, const float* x, int64_t B, float* out) {
    or_kfftr_cfg* f = or_kfftr_alloc(nfft, 0);
    for (int64_t b = 0; b < B; ++b) or_adapter_forward(f, nfft, x + (size_t)b * nfft, out + (size_t)b * (nfft + 2));
    or_kfftr_free(f);
}

/* kernels_benchmark.cc / micro_kernels_benchmark.cc: `reps` calls of one scalar
 * kernel (kernels.cc:18-36) on n elements (op 0 axpy, 1 axpy_windowed,
 * 2 normalize_and_clear); the caller times the call. */
void or_bench_kernel(int op, size_t n, int64_t reps, float* dst, const float* src, const float* win,
                     float* out) {
    for (int64_t r = 0; r < reps; ++r) {
        if (op == 0)
            or_axpy(dst, src, 0.5f, n);
        else if (op == 1)
            or_axpy_windowed(dst, src, win, 0.5f, n);
        else
            or_normalize_and_clear(out, dst, win, 1e-8f, n);
    }
}
