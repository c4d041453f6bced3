/*
 * ORACLE -- test infrastructure only.  See pgo_oracle.h for the contract.
 *
 * CPU restatement of the reference path:
 *   graph.cpp:27-113   factor construction: PriorFactor<Pose2> on the first key,
 *                      BetweenFactor<Pose2>(id_1, id_2, delta, Covariance(Q)),
 *                      Q from the row-major float64[9] (graph.hpp:45-58)
 *   graph.cpp:119      LevenbergMarquardtOptimizer(graph, initial).optimize()
 *   graph.cpp:122-130  write-back of x, y, theta
 *
 * GTSAM 4.0.x semantics restated (GTSAM is absent):
 *   Rot2::normalize (|c^2+s^2-1| > 1e-10 -> scale by (c^2+s^2)^-1/2);
 *   Pose2::between + closed-form H1, H2 = I; default Pose2 chart
 *   (Local = (x, y, theta), Retract(v) = p * Pose2(v)); BetweenFactor
 *   e = Local(z, between(p1,p2)); PriorFactor e = -Local(x, prior), H = I;
 *   Gaussian::Covariance smart diagonal check (1e-9) else Omega = lower(Q^-1)
 *   mirrored (LLT reads the lower triangle); LM tryLambda / decreaseLambda /
 *   increaseLambda and NonlinearOptimizer::checkConvergence with GTSAM defaults.
 *
 * Linear solver: GTSAM recomputes a COLAMD ordering and runs multifrontal
 * Cholesky each solve.  Here: approximate-minimum-degree ordering on the pose
 * graph (computed once per graph -- an advantage to this CPU baseline), relaxed
 * supernodes, multifrontal numeric factorisation with blocked dense kernels
 * (OpenMP across front columns), supernodal triangular solves.  Any exact
 * direct method gives GTSAM's delta up to rounding.
 */
#include "pgo_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  double x, y, c, s;
} pose2;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ------------------------------------------------------------ Pose2 algebra */
static inline void rot_normalize(double *c, double *s) { /* GTSAM Rot2::normalize */
  double scale = (*c) * (*c) + (*s) * (*s);
  if (fabs(scale - 1.0) > 1e-10) {
    double f = pow(scale, -0.5);
    *c *= f;
    *s *= f;
  }
}

static inline pose2 pose_from_xyt(const double *v) { /* Pose2(x,y,theta): Rot2::fromAngle */
  pose2 p = {v[0], v[1], cos(v[2]), sin(v[2])};
  return p;
}

static inline pose2 between(pose2 a, pose2 b) { /* GTSAM Pose2::between */
  pose2 r;
  r.c = a.c * b.c + a.s * b.s;
  r.s = -a.s * b.c + a.c * b.s;
  rot_normalize(&r.c, &r.s);
  double dx = b.x - a.x, dy = b.y - a.y;
  r.x = a.c * dx + a.s * dy;
  r.y = -a.s * dx + a.c * dy;
  return r;
}

static inline void local3(pose2 a, pose2 b, double *e) { /* Local(a, b), default chart */
  pose2 d = between(a, b);
  e[0] = d.x;
  e[1] = d.y;
  e[2] = atan2(d.s, d.c);
}

static inline pose2 retract(pose2 p, const double *d) { /* p * Pose2(d0, d1, d2) */
  double cd = cos(d[2]), sd = sin(d[2]);
  pose2 r;
  r.c = p.c * cd - p.s * sd;
  r.s = p.s * cd + p.c * sd;
  rot_normalize(&r.c, &r.s);
  r.x = p.x + p.c * d[0] - p.s * d[1];
  r.y = p.y + p.s * d[0] + p.c * d[1];
  return r;
}

/* ------------------------------------------------------------- noise model */
int orc_information(const double *q, double *om) {
  int full = 0;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      if (i != j && fabs(q[3 * i + j]) > 1e-9) full = 1;
  if (!full) { /* Diagonal::Variances */
    memset(om, 0, 9 * sizeof(double));
    for (int i = 0; i < 3; i++) {
      double v = q[4 * i];
      if (!(v > 0.0) || !isfinite(v)) return ORC_E_BAD_COV;
      om[4 * i] = 1.0 / v;
    }
    return ORC_OK;
  }
  /* Information(Q.inverse()): Eigen 3x3 inverse via cofactors */
  double a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5], g = q[6], h = q[7], k = q[8];
  double A = e * k - f * h, B = -(d * k - f * g), C = d * h - e * g;
  double det = a * A + b * B + c * C;
  if (!(fabs(det) > 0.0) || !isfinite(det)) return ORC_E_BAD_COV;
  double inv[9] = {A / det, -(b * k - c * h) / det, (b * f - c * e) / det,
                   B / det, (a * k - c * g) / det,  -(a * f - c * d) / det,
                   C / det, -(a * h - b * g) / det, (a * e - b * d) / det};
  /* LLT reads the lower triangle: Omega = lower(inv) mirrored */
  for (int i = 0; i < 3; i++)
    for (int j = 0; j <= i; j++) om[3 * i + j] = om[3 * j + i] = inv[3 * i + j];
  /* positive definiteness (LLT success) */
  double l00 = om[0];
  if (!(l00 > 0)) return ORC_E_BAD_COV;
  l00 = sqrt(l00);
  double l10 = om[3] / l00, l20 = om[6] / l00;
  double l11 = om[4] - l10 * l10;
  if (!(l11 > 0)) return ORC_E_BAD_COV;
  l11 = sqrt(l11);
  double l21 = (om[7] - l20 * l10) / l11;
  double l22 = om[8] - l20 * l20 - l21 * l21;
  if (!(l22 > 0)) return ORC_E_BAD_COV;
  return ORC_OK;
}

/* ------------------------------------------------------------- dyn int vec */
typedef struct {
  int *a;
  int n, cap;
} ivec;
static void iv_push(ivec *v, int x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? 2 * v->cap : 4;
    v->a = (int *)realloc(v->a, (size_t)v->cap * sizeof(int));
  }
  v->a[v->n++] = x;
}
static void iv_free(ivec *v) {
  free(v->a);
  v->a = NULL;
  v->n = v->cap = 0;
}

/* ------------------------------------------------- approximate min degree
 * Quotient-graph minimum degree with AMD-style approximate external degrees
 * (Amestoy, Davis & Duff 1996): elements absorb their neighbours on
 * elimination, |Le \ Lp| via the w(e) trick, aggressive absorption. */
static void amd_order(int n, const int *xadj, const int *adj, int *perm) {
  ivec *av = (ivec *)calloc(n, sizeof(ivec)), *ae = (ivec *)calloc(n, sizeof(ivec));
  ivec *le = (ivec *)calloc(n, sizeof(ivec));
  char *status = (char *)calloc(n, 1); /* 0 var, 1 element, 2 absorbed */
  int *deg = (int *)malloc(n * sizeof(int)), *w = (int *)malloc(n * sizeof(int));
  int *wtag = (int *)malloc(n * sizeof(int)), *mark = (int *)malloc(n * sizeof(int));
  int *head = (int *)malloc((n + 1) * sizeof(int)), *next = (int *)malloc(n * sizeof(int));
  int *prev = (int *)malloc(n * sizeof(int));
  for (int i = 0; i <= n; i++) head[i] = -1;
  for (int i = 0; i < n; i++) wtag[i] = mark[i] = -1;
#define BK_INS(i, d)                       \
  do {                                     \
    next[i] = head[d];                     \
    prev[i] = -1;                          \
    if (head[d] >= 0) prev[head[d]] = (i); \
    head[d] = (i);                         \
  } while (0)
#define BK_DEL(i)                                \
  do {                                           \
    if (prev[i] >= 0) next[prev[i]] = next[i];   \
    else head[deg[i]] = next[i];                 \
    if (next[i] >= 0) prev[next[i]] = prev[i];   \
  } while (0)
  for (int i = 0; i < n; i++) {
    for (int k = xadj[i]; k < xadj[i + 1]; k++)
      if (adj[k] != i) iv_push(&av[i], adj[k]);
    deg[i] = av[i].n;
  }
  for (int i = n - 1; i >= 0; i--) BK_INS(i, deg[i]);
  int mindeg = 0;
  for (int k = 0; k < n; k++) {
    while (head[mindeg] < 0) mindeg++;
    int p = head[mindeg];
    BK_DEL(p);
    perm[k] = p;
    ivec lp = {0, 0, 0};
    mark[p] = k;
    for (int t = 0; t < av[p].n; t++) {
      int j = av[p].a[t];
      if (status[j] == 0 && mark[j] != k) {
        mark[j] = k;
        iv_push(&lp, j);
      }
    }
    for (int t = 0; t < ae[p].n; t++) {
      int e = ae[p].a[t];
      if (status[e] != 1) continue;
      for (int u = 0; u < le[e].n; u++) {
        int j = le[e].a[u];
        if (status[j] == 0 && mark[j] != k) {
          mark[j] = k;
          iv_push(&lp, j);
        }
      }
      status[e] = 2;
      iv_free(&le[e]);
    }
    status[p] = 1;
    iv_free(&av[p]);
    iv_free(&ae[p]);
    le[p] = lp;
    for (int t = 0; t < lp.n; t++) BK_DEL(lp.a[t]);
    for (int t = 0; t < lp.n; t++) {
      int i = lp.a[t];
      for (int u = 0; u < ae[i].n; u++) {
        int e = ae[i].a[u];
        if (status[e] != 1) continue;
        if (wtag[e] != k) {
          wtag[e] = k;
          w[e] = le[e].n;
        }
        w[e]--;
      }
    }
    int nleft = n - k - 1;
    for (int t = 0; t < lp.n; t++) {
      int i = lp.a[t];
      long dext = 0;
      int m = 0;
      for (int u = 0; u < ae[i].n; u++) {
        int e = ae[i].a[u];
        if (status[e] != 1) continue;
        if (w[e] == 0) { /* aggressive absorption: Le subset of Lp */
          status[e] = 2;
          iv_free(&le[e]);
          continue;
        }
        ae[i].a[m++] = e;
        dext += w[e];
      }
      ae[i].n = m;
      iv_push(&ae[i], p);
      m = 0;
      for (int u = 0; u < av[i].n; u++) {
        int j = av[i].a[u];
        if (status[j] == 0 && mark[j] != k) av[i].a[m++] = j;
      }
      av[i].n = m;
      long d = (long)av[i].n + (lp.n - 1) + dext;
      long bound = (long)deg[i] + lp.n - 1;
      if (d > bound) d = bound;
      if (d > nleft - 1) d = nleft - 1;
      if (d < 0) d = 0;
      deg[i] = (int)d;
      BK_INS(i, deg[i]);
      if (deg[i] < mindeg) mindeg = deg[i];
    }
  }
#undef BK_INS
#undef BK_DEL
  for (int i = 0; i < n; i++) {
    iv_free(&av[i]);
    iv_free(&ae[i]);
    iv_free(&le[i]);
  }
  free(av);
  free(ae);
  free(le);
  free(status);
  free(deg);
  free(w);
  free(wtag);
  free(mark);
  free(head);
  free(next);
  free(prev);
}

/* -------------------------------------------------------- symbolic analysis */
typedef struct {
  int n;          /* poses */
  int *perm;      /* new -> old */
  int *iperm;     /* old -> new */
  int ns;         /* supernodes */
  int *sfirst;    /* [ns+1] pose columns (new index) */
  int *rptr;      /* [ns+1] */
  int *rows;      /* below-diagonal pose rows, sorted (new index) */
  int *sparent;   /* supernodal etree */
  int *nchild;
  size_t *loff;   /* [ns+1] offset of each scalar panel (3m x 3w, column-major) */
  int *acol;      /* [n+1] per new column pose: assembly list */
  int *aent;      /* edge id; >= 0: block B_e at (row=iperm[ej]... see fill); encoded */
  int *arow;      /* row pose (new) of each assembly entry */
  double flops;
  double nnzl;
  int maxfront;   /* max scalar front size */
} chol_sym;

static void sym_free(chol_sym *s) {
  if (!s) return;
  free(s->perm);
  free(s->iperm);
  free(s->sfirst);
  free(s->rptr);
  free(s->rows);
  free(s->sparent);
  free(s->nchild);
  free(s->loff);
  free(s->acol);
  free(s->aent);
  free(s->arow);
  free(s);
}

static int cmp_int(const void *a, const void *b) {
  int x = *(const int *)a, y = *(const int *)b;
  return (x > y) - (x < y);
}

/* order_in (optional, new -> old pose index): a fill-reducing ordering given
 * by the caller instead of AMD -- bench.py times the CPU path on the same
 * nested-dissection permutation the GPU plan uses, so the two factorisations
 * have identical fill and flops */
static chol_sym *sym_analyze(int n, int ne, const int32_t *ei, const int32_t *ej, const int32_t *order_in) {
  chol_sym *S = (chol_sym *)calloc(1, sizeof(chol_sym));
  S->n = n;
  /* pose adjacency (old index), deduplicated */
  int *cnt = (int *)calloc(n + 1, sizeof(int));
  for (int e = 0; e < ne; e++)
    if (ei[e] != ej[e]) {
      cnt[ei[e]]++;
      cnt[ej[e]]++;
    }
  int *xadj = (int *)malloc((n + 1) * sizeof(int));
  xadj[0] = 0;
  for (int i = 0; i < n; i++) xadj[i + 1] = xadj[i] + cnt[i];
  int *adj = (int *)malloc((size_t)(xadj[n] > 0 ? xadj[n] : 1) * sizeof(int));
  int *fill = (int *)malloc(n * sizeof(int));
  memcpy(fill, xadj, n * sizeof(int));
  for (int e = 0; e < ne; e++)
    if (ei[e] != ej[e]) {
      adj[fill[ei[e]]++] = ej[e];
      adj[fill[ej[e]]++] = ei[e];
    }
  /* dedupe */
  int *mark = (int *)malloc(n * sizeof(int));
  for (int i = 0; i < n; i++) mark[i] = -1;
  int *xa2 = (int *)malloc((n + 1) * sizeof(int));
  int w = 0;
  for (int i = 0; i < n; i++) {
    xa2[i] = w;
    for (int k = xadj[i]; k < xadj[i + 1]; k++) {
      int j = adj[k];
      if (mark[j] != i) {
        mark[j] = i;
        adj[w++] = j;
      }
    }
  }
  xa2[n] = w;
  free(xadj);
  xadj = xa2;

  int *perm0 = (int *)malloc(n * sizeof(int));
  if (order_in) memcpy(perm0, order_in, n * sizeof(int));
  else amd_order(n, xadj, adj, perm0);
  int *ip0 = (int *)malloc(n * sizeof(int));
  for (int k = 0; k < n; k++) ip0[perm0[k]] = k;

  /* elimination tree of the permuted pattern (Liu, path compression) */
  int *parent = (int *)malloc(n * sizeof(int)), *anc = (int *)malloc(n * sizeof(int));
  for (int j = 0; j < n; j++) {
    parent[j] = -1;
    anc[j] = -1;
    int oj = perm0[j];
    for (int k = xadj[oj]; k < xadj[oj + 1]; k++) {
      int i = ip0[adj[k]];
      if (i >= j) continue;
      int r = i;
      while (anc[r] != -1 && anc[r] != j) {
        int t = anc[r];
        anc[r] = j;
        r = t;
      }
      if (anc[r] == -1) {
        anc[r] = j;
        parent[r] = j;
      }
    }
  }
  /* postorder (iterative DFS; children visited in increasing order) */
  int *chead = (int *)malloc(n * sizeof(int)), *cnext = (int *)malloc(n * sizeof(int));
  for (int j = 0; j < n; j++) chead[j] = -1;
  for (int j = n - 1; j >= 0; j--)
    if (parent[j] >= 0) {
      cnext[j] = chead[parent[j]];
      chead[parent[j]] = j;
    }
  int *post = (int *)malloc(n * sizeof(int)), *stk = (int *)malloc(n * sizeof(int));
  int np = 0;
  for (int r = 0; r < n; r++) {
    if (parent[r] != -1) continue;
    int top = 0;
    stk[0] = r;
    while (top >= 0) {
      int j = stk[top];
      int c = chead[j];
      if (c == -1) {
        top--;
        post[np++] = j;
      } else {
        chead[j] = cnext[c];
        stk[++top] = c;
      }
    }
  }
  free(chead);
  free(cnext);
  S->perm = (int *)malloc(n * sizeof(int));
  S->iperm = (int *)malloc(n * sizeof(int));
  int *pold = (int *)malloc(n * sizeof(int)); /* post position of old etree node */
  for (int k = 0; k < n; k++) {
    S->perm[k] = perm0[post[k]];
    pold[post[k]] = k;
  }
  for (int k = 0; k < n; k++) S->iperm[S->perm[k]] = k;
  int *par = (int *)malloc(n * sizeof(int));
  for (int k = 0; k < n; k++) par[k] = parent[post[k]] >= 0 ? pold[parent[post[k]]] : -1;
  free(perm0);
  free(ip0);
  free(parent);
  free(anc);
  free(post);
  free(pold);
  free(stk);

  /* column counts (off-diagonal pose rows per column) via row subtrees */
  int *cc = (int *)calloc(n, sizeof(int));
  for (int i = 0; i < n; i++) mark[i] = -1;
  for (int i = 0; i < n; i++) {
    mark[i] = i;
    int oi = S->perm[i];
    for (int k = xadj[oi]; k < xadj[oi + 1]; k++) {
      int j = S->iperm[adj[k]];
      if (j >= i) continue;
      while (mark[j] != i) {
        cc[j]++;
        mark[j] = i;
        j = par[j];
      }
    }
  }
  /* number of etree children */
  int *nch = (int *)calloc(n, sizeof(int));
  for (int j = 0; j < n; j++)
    if (par[j] >= 0) nch[par[j]]++;
  /* fundamental supernodes */
  int *sf = (int *)malloc((n + 1) * sizeof(int));
  int ns0 = 0;
  for (int j = 0; j < n; j++) {
    if (j > 0 && par[j - 1] == j && nch[j] == 1 && cc[j - 1] == cc[j] + 1) continue;
    sf[ns0++] = j;
  }
  sf[ns0] = n;
  /* relaxed amalgamation: merge a child that immediately precedes its parent
   * when the explicit zeros it introduces are few (CHOLMOD-like thresholds). */
  int *of = (int *)malloc((ns0 + 1) * sizeof(int)); /* output first cols */
  double *onz = (double *)malloc((ns0 + 1) * sizeof(double)); /* true nnz */
  int *onb = (int *)malloc((ns0 + 1) * sizeof(int));          /* below rows */
  int *ol = (int *)malloc((ns0 + 1) * sizeof(int));           /* last col + 1 */
  int no = 0;
  for (int s = 0; s < ns0; s++) {
    int f = sf[s], l = sf[s + 1];
    int wdt = l - f;
    int nb = cc[l - 1];
    double nz = 0.5 * wdt * (wdt + 1.0) + (double)wdt * nb;
    while (no > 0) {
      int t = no - 1;
      if (ol[t] != f) break;
      int lastc = ol[t] - 1;
      if (par[lastc] < f || par[lastc] >= l) break;
      int W = (l - of[t]);
      double tot = 0.5 * W * (W + 1.0) + (double)W * nb;
      double tnz = nz + onz[t];
      double z = (tot - tnz) / tot;
      int ok = (W <= 2) || (W <= 6 && z < 0.8) || (W <= 16 && z < 0.1) || (z < 0.05);
      if (!ok) break;
      f = of[t];
      nz = tnz;
      no--;
    }
    of[no] = f;
    ol[no] = l;
    onz[no] = nz;
    onb[no] = nb;
    no++;
  }
  S->ns = no;
  S->sfirst = (int *)malloc((no + 1) * sizeof(int));
  for (int s = 0; s < no; s++) S->sfirst[s] = of[s];
  S->sfirst[no] = n;
  free(sf);
  free(of);
  free(onz);
  free(onb);
  free(ol);
  free(cc);
  free(nch);
  /* supernode of each column */
  int *snode = (int *)malloc(n * sizeof(int));
  for (int s = 0; s < no; s++)
    for (int j = S->sfirst[s]; j < S->sfirst[s + 1]; j++) snode[j] = s;
  S->sparent = (int *)malloc(no * sizeof(int));
  S->nchild = (int *)calloc(no, sizeof(int));
  for (int s = 0; s < no; s++) {
    int lc = S->sfirst[s + 1] - 1;
    S->sparent[s] = par[lc] >= 0 ? snode[par[lc]] : -1;
    if (S->sparent[s] >= 0) S->nchild[S->sparent[s]]++;
  }
  /* below-diagonal row structure per supernode: A's rows below + children's rows */
  S->rptr = (int *)malloc((no + 1) * sizeof(int));
  ivec *rl = (ivec *)calloc(no, sizeof(ivec));
  int *cheadS = (int *)malloc(no * sizeof(int)), *cnextS = (int *)malloc(no * sizeof(int));
  for (int s = 0; s < no; s++) cheadS[s] = -1;
  for (int s = no - 1; s >= 0; s--)
    if (S->sparent[s] >= 0) {
      cnextS[s] = cheadS[S->sparent[s]];
      cheadS[S->sparent[s]] = s;
    }
  for (int i = 0; i < n; i++) mark[i] = -1;
  long total = 0;
  for (int s = 0; s < no; s++) {
    int f = S->sfirst[s], l = S->sfirst[s + 1];
    for (int j = f; j < l; j++) {
      int oj = S->perm[j];
      for (int k = xadj[oj]; k < xadj[oj + 1]; k++) {
        int i = S->iperm[adj[k]];
        if (i >= l && mark[i] != s) {
          mark[i] = s;
          iv_push(&rl[s], i);
        }
      }
    }
    for (int c = cheadS[s]; c >= 0; c = cnextS[c]) {
      for (int t = 0; t < rl[c].n; t++) {
        int i = rl[c].a[t];
        if (i >= l && mark[i] != s) {
          mark[i] = s;
          iv_push(&rl[s], i);
        }
      }
    }
    if (rl[s].n > 1) qsort(rl[s].a, rl[s].n, sizeof(int), cmp_int);   /* (a root's list is empty: a == NULL) */
    total += rl[s].n;
  }
  S->rows = (int *)malloc((size_t)(total > 0 ? total : 1) * sizeof(int));
  S->loff = (size_t *)malloc((no + 1) * sizeof(size_t));
  size_t off = 0;
  long pos = 0;
  double flops = 0, nnzl = 0;
  int maxfront = 0;
  for (int s = 0; s < no; s++) {
    S->rptr[s] = (int)pos;
    if (rl[s].n) memcpy(S->rows + pos, rl[s].a, rl[s].n * sizeof(int));
    pos += rl[s].n;
    int wd = 3 * (S->sfirst[s + 1] - S->sfirst[s]);
    int m = wd + 3 * rl[s].n;
    S->loff[s] = off;
    off += (size_t)m * wd;
    if (m > maxfront) maxfront = m;
    /* flops of partial factorisation of an m x m front on its first wd columns */
    for (int k = 0; k < wd; k++) {
      double r = m - k - 1;
      flops += 1 + r + r * (r + 1); /* sqrt/div, scale, rank-1 update (lower) */
      nnzl += r + 1;
    }
    iv_free(&rl[s]);
  }
  S->rptr[no] = (int)pos;
  S->loff[no] = off;
  S->flops = flops;
  S->nnzl = nnzl;
  S->maxfront = maxfront;
  free(rl);
  free(cheadS);
  free(cnextS);
  free(snode);
  free(par);
  /* assembly lists: each between factor's off-diagonal block goes to column
   * min(new i, new j), row max(...).  aent = e (block B_e rows=ei) or ~e
   * (transposed: rows = ej). */
  S->acol = (int *)calloc(n + 1, sizeof(int));
  for (int e = 0; e < ne; e++) {
    if (ei[e] == ej[e]) continue;
    int a = S->iperm[ei[e]], b = S->iperm[ej[e]];
    S->acol[(a < b ? a : b) + 1]++;
  }
  for (int j = 0; j < n; j++) S->acol[j + 1] += S->acol[j];
  int na = S->acol[n];
  S->aent = (int *)malloc((na > 0 ? na : 1) * sizeof(int));
  S->arow = (int *)malloc((na > 0 ? na : 1) * sizeof(int));
  memcpy(fill, S->acol, n * sizeof(int));
  for (int e = 0; e < ne; e++) {
    if (ei[e] == ej[e]) continue;
    int a = S->iperm[ei[e]], b = S->iperm[ej[e]];
    int col = a < b ? a : b, row = a < b ? b : a;
    int slot = fill[col]++;
    S->aent[slot] = (row == a) ? e : ~e; /* row pose is ei -> B_e, else B_e^T */
    S->arow[slot] = row;
  }
  free(fill);
  free(mark);
  free(cnt);
  free(xadj);
  free(adj);
  return S;
}

/* ------------------------------------------------------------ dense kernels
 * Column-major, leading dimension ld.  The Schur update C -= A A^T (lower) is
 * register-tiled 8x4 with GCC vector extensions (AVX2/FMA under x86-64-v3). */
typedef double v4d __attribute__((vector_size(32)));

static void syrk_lower(int m, int kk, const double *A, int lda, double *C, int ldc) {
  /* C[i][j] -= sum_k A[i][k] A[j][k] for i >= j, 0 <= i,j < m */
  int nj = (m + 3) / 4;
#pragma omp parallel for schedule(dynamic, 1) if ((double)m * m * kk > 4e6)
  for (int jb = 0; jb < nj; jb++) {
    int j0 = jb * 4;
    int jw = m - j0 < 4 ? m - j0 : 4;
    /* diagonal tile region rows j0..j0+3 handled scalar */
    for (int j = j0; j < j0 + jw; j++)
      for (int i = j; i < j0 + jw; i++) {
        double acc = 0;
        for (int k = 0; k < kk; k++) acc += A[i + (size_t)k * lda] * A[j + (size_t)k * lda];
        C[i + (size_t)j * ldc] -= acc;
      }
    int i0 = j0 + jw;
    if (jw == 4) {
      int i = i0;
      for (; i + 8 <= m; i += 8) {
        v4d c00 = {0}, c01 = {0}, c10 = {0}, c11 = {0}, c20 = {0}, c21 = {0}, c30 = {0}, c31 = {0};
        for (int k = 0; k < kk; k++) {
          const double *ak = A + (size_t)k * lda;
          v4d a0, a1;
          memcpy(&a0, ak + i, 32);
          memcpy(&a1, ak + i + 4, 32);
          double b0 = ak[j0], b1 = ak[j0 + 1], b2 = ak[j0 + 2], b3 = ak[j0 + 3];
          c00 += a0 * b0;
          c01 += a1 * b0;
          c10 += a0 * b1;
          c11 += a1 * b1;
          c20 += a0 * b2;
          c21 += a1 * b2;
          c30 += a0 * b3;
          c31 += a1 * b3;
        }
        double *cj;
        v4d t;
        cj = C + (size_t)j0 * ldc + i;
        memcpy(&t, cj, 32); t -= c00; memcpy(cj, &t, 32);
        memcpy(&t, cj + 4, 32); t -= c01; memcpy(cj + 4, &t, 32);
        cj += ldc;
        memcpy(&t, cj, 32); t -= c10; memcpy(cj, &t, 32);
        memcpy(&t, cj + 4, 32); t -= c11; memcpy(cj + 4, &t, 32);
        cj += ldc;
        memcpy(&t, cj, 32); t -= c20; memcpy(cj, &t, 32);
        memcpy(&t, cj + 4, 32); t -= c21; memcpy(cj + 4, &t, 32);
        cj += ldc;
        memcpy(&t, cj, 32); t -= c30; memcpy(cj, &t, 32);
        memcpy(&t, cj + 4, 32); t -= c31; memcpy(cj + 4, &t, 32);
      }
      i0 = i;
    }
    for (int j = j0; j < j0 + jw; j++)
      for (int i = i0; i < m; i++) {
        double acc = 0;
        for (int k = 0; k < kk; k++) acc += A[i + (size_t)k * lda] * A[j + (size_t)k * lda];
        C[i + (size_t)j * ldc] -= acc;
      }
  }
}

/* Partial Cholesky of the m x m lower front F (ld m) on its first w columns;
 * leaves L11, L21 in F[:, :w] and the Schur complement in F[w:, w:].
 * Returns 0 or -1 on a non-positive / non-finite pivot. */
#define NB 48
/* Rows [r0, m) of the panel columns [kb, kb + nb) once the panel's diagonal
 * block is factored: L21 = A21 L11^-T, column by column (left-looking inside
 * the panel), in 64-row blocks spread over the threads.  Every element sees
 * the same operations in the same order as a column sweep over all rows. */
static void panel_trsm(double *F, int m, int kb, int nb, int r0) {
  const int nblk = (m - r0 + 63) / 64;
#pragma omp parallel for schedule(dynamic, 1) if ((double)(m - r0) * nb * nb > 1e6)
  for (int bi = 0; bi < nblk; bi++) {
    const int i0 = r0 + 64 * bi, i1 = i0 + 64 < m ? i0 + 64 : m;
    for (int k = kb; k < kb + nb; k++) {
      double *colk = F + (size_t)k * m;
      for (int t = kb; t < k; t++) {
        const double ljk = F[k + (size_t)t * m];
        const double *colt = F + (size_t)t * m;
        for (int i = i0; i < i1; i++) colk[i] -= colt[i] * ljk;
      }
      const double inv = 1.0 / colk[k];
      for (int i = i0; i < i1; i++) colk[i] *= inv;
    }
  }
}

static int front_factor(double *F, int m, int w) {
  for (int kb = 0; kb < w; kb += NB) {
    int nb = w - kb < NB ? w - kb : NB;
    const int r0 = kb + nb;
    /* unblocked on the panel's diagonal block (left-looking inside the panel) */
    for (int k = kb; k < r0; k++) {
      double *colk = F + (size_t)k * m;
      for (int t = kb; t < k; t++) {
        double ljk = F[k + (size_t)t * m];
        const double *colt = F + (size_t)t * m;
        for (int i = k; i < r0; i++) colk[i] -= colt[i] * ljk;
      }
      double d = colk[k];
      if (!(d > 0.0) || !isfinite(d)) return -1;
      d = sqrt(d);
      colk[k] = d;
      double inv = 1.0 / d;
      for (int i = k + 1; i < r0; i++) colk[i] *= inv;
    }
    /* the rows below it, then the trailing update (lower part) */
    if (r0 < m) {
      panel_trsm(F, m, kb, nb, r0);
      syrk_lower(m - r0, nb, F + r0 + (size_t)kb * m, m, F + r0 + (size_t)r0 * m, m);
    }
  }
  return 0;
}

/* ------------------------------------------------------------ numeric */
typedef struct {
  chol_sym *S;
  double *L;      /* panels */
  double **U;     /* [ns] update matrix of each front until its parent consumed it */
  int *cptr, *child; /* children of each supernode, increasing */
  int nlev;
  int *lptr, *lfront; /* fronts by height (leaves first), largest first within a level */
} chol_num;

static double front_work(const chol_sym *S, int s) {
  double wd = 3.0 * (S->sfirst[s + 1] - S->sfirst[s]), m = wd + 3.0 * (S->rptr[s + 1] - S->rptr[s]);
  return wd * m * m;
}

static chol_num *num_create(chol_sym *S) {
  chol_num *N = (chol_num *)calloc(1, sizeof(chol_num));
  N->S = S;
  int ns = S->ns;
  N->L = (double *)malloc((S->loff[ns] > 0 ? S->loff[ns] : 1) * sizeof(double));
  N->U = (double **)calloc(ns > 0 ? ns : 1, sizeof(double *));
  N->cptr = (int *)calloc(ns + 1, sizeof(int));
  N->child = (int *)malloc((ns > 0 ? ns : 1) * sizeof(int));
  for (int s = 0; s < ns; s++)
    if (S->sparent[s] >= 0) N->cptr[S->sparent[s] + 1]++;
  for (int s = 0; s < ns; s++) N->cptr[s + 1] += N->cptr[s];
  int *fill = (int *)malloc((ns + 1) * sizeof(int));
  memcpy(fill, N->cptr, (ns + 1) * sizeof(int));
  for (int s = 0; s < ns; s++)
    if (S->sparent[s] >= 0) N->child[fill[S->sparent[s]]++] = s;
  /* heights (children precede parents in the postorder) */
  int *h = (int *)calloc(ns > 0 ? ns : 1, sizeof(int));
  int nlev = 0;
  for (int s = 0; s < ns; s++) {
    if (S->sparent[s] >= 0 && h[S->sparent[s]] < h[s] + 1) h[S->sparent[s]] = h[s] + 1;
    if (h[s] + 1 > nlev) nlev = h[s] + 1;
  }
  N->nlev = nlev;
  N->lptr = (int *)calloc(nlev + 1, sizeof(int));
  N->lfront = (int *)malloc((ns > 0 ? ns : 1) * sizeof(int));
  for (int s = 0; s < ns; s++) N->lptr[h[s] + 1]++;
  for (int l = 0; l < nlev; l++) N->lptr[l + 1] += N->lptr[l];
  memcpy(fill, N->lptr, (nlev + 1) * sizeof(int));
  for (int s = 0; s < ns; s++) N->lfront[fill[h[s]]++] = s;
  for (int l = 0; l < nlev; l++) { /* largest first (insertion sort is fine: levels are small or cheap) */
    int a = N->lptr[l], b = N->lptr[l + 1];
    for (int i = a + 1; i < b; i++) {
      int x = N->lfront[i], j = i - 1;
      double wx = front_work(S, x);
      while (j >= a && front_work(S, N->lfront[j]) < wx) {
        N->lfront[j + 1] = N->lfront[j];
        j--;
      }
      N->lfront[j + 1] = x;
    }
  }
  free(fill);
  free(h);
  return N;
}
static void num_free(chol_num *N) {
  if (!N) return;
  free(N->L);
  if (N->U)
    for (int s = 0; s < N->S->ns; s++) free(N->U[s]);
  free(N->U);
  free(N->cptr);
  free(N->child);
  free(N->lptr);
  free(N->lfront);
  free(N);
}

/* One front: assemble A's entries (+lam), extend-add the children's update
 * matrices in increasing child order, partial Cholesky, keep the panel, keep
 * the update matrix for the parent.  rel: per-thread scratch of n ints. */
static int factor_one(chol_num *N, int s, const double *hdiag, const double *hoff, double lam, int *rel) {
  chol_sym *S = N->S;
  int f = S->sfirst[s], l = S->sfirst[s + 1];
  int wp = l - f, nb = S->rptr[s + 1] - S->rptr[s];
  const int *R = S->rows + S->rptr[s];
  int m = 3 * (wp + nb), wd = 3 * wp;
  /* a big front (run alone, see num_factor) is zeroed, extended and copied out
   * by all the threads; the small ones by their own thread */
  const int par = (double)wd * m * m > 2e7 && !omp_in_parallel();
  double *F = (double *)malloc((size_t)m * m > 0 ? (size_t)m * m * sizeof(double) : sizeof(double));
#pragma omp parallel for schedule(static) if (par)
  for (int j = 0; j < m; j++) memset(F + (size_t)j * m, 0, (size_t)m * sizeof(double));
  for (int j = f; j < l; j++) rel[j] = j - f;
  for (int t = 0; t < nb; t++) rel[R[t]] = wp + t;
  for (int j = f; j < l; j++) {
    int lj = 3 * (j - f);
    const double *D = hdiag + 9 * (size_t)S->perm[j];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b <= a; b++) F[(lj + a) + (size_t)(lj + b) * m] += D[3 * a + b];
    for (int a = 0; a < 3; a++) F[(lj + a) + (size_t)(lj + a) * m] += lam;
    for (int q = S->acol[j]; q < S->acol[j + 1]; q++) {
      int code = S->aent[q];
      int e = code >= 0 ? code : ~code;
      const double *B = hoff + 9 * (size_t)e;
      int li = 3 * rel[S->arow[q]];
      if (code >= 0) /* rows = ei, cols = ej: block B */
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) F[(li + a) + (size_t)(lj + b) * m] += B[3 * a + b];
      else /* rows = ej, cols = ei: block B^T */
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) F[(li + a) + (size_t)(lj + b) * m] += B[3 * b + a];
    }
  }
  for (int q = N->cptr[s]; q < N->cptr[s + 1]; q++) {
    int cs = N->child[q];
    const int *Rc = S->rows + S->rptr[cs];
    int nbc = S->rptr[cs + 1] - S->rptr[cs];
    int mc = 3 * nbc;
    const double *U = N->U[cs];
    if (U)
#pragma omp parallel for schedule(dynamic, 8) if (par)
      for (int b = 0; b < nbc; b++) {   /* (b, y): column gb + y of F, one thread's */
        int gb = 3 * rel[Rc[b]];
        for (int y = 0; y < 3; y++) {
          int colU = 3 * b + y;
          double *Fc = F + (size_t)(gb + y) * m;
          const double *Uc = U + (size_t)colU * mc;
          for (int a = b; a < nbc; a++) {
            int ga = 3 * rel[Rc[a]];
            for (int x = (a == b ? y : 0); x < 3; x++) Fc[ga + x] += Uc[3 * a + x];
          }
        }
      }
    free(N->U[cs]);
    N->U[cs] = NULL;
  }
  int rc = front_factor(F, m, wd) != 0 ? ORC_E_INDETERMINANT : ORC_OK;
  if (rc == ORC_OK) {
    double *Ls = N->L + S->loff[s];
#pragma omp parallel for schedule(static) if (par)
    for (int j = 0; j < wd; j++) memcpy(Ls + (size_t)j * m, F + (size_t)j * m, (size_t)m * sizeof(double));
    int mu = m - wd;
    if (S->sparent[s] >= 0 && mu > 0) {
      double *U = (double *)malloc((size_t)mu * mu * sizeof(double));
#pragma omp parallel for schedule(static) if (par)
      for (int j = 0; j < mu; j++) memcpy(U + (size_t)j * mu, F + wd + (size_t)(wd + j) * m, mu * sizeof(double));
      N->U[s] = U;
    }
  }
  free(F);
  return rc;
}

/* Factor H + lam I given per-pose diagonal blocks (old index, 9 row-major) and
 * per-edge off-diagonal blocks B_e = H_{ei,ej} (9 row-major).  Level by level
 * (leaves first): the fronts of a level in parallel, one thread each, except
 * the large fronts, which run one at a time with the Schur updates spread over
 * the threads.  Every front sums its children in increasing order and every
 * Schur-update element is one thread's fixed-order dot product, so the result
 * does not depend on the thread count. */
static int num_factor(chol_num *N, const double *hdiag, const double *hoff, double lam) {
  chol_sym *S = N->S;
  int rc = ORC_OK;
  const double big = 2e7;   /* flops: above this a front gets all the threads */
  int *rel0 = (int *)malloc((S->n > 0 ? S->n : 1) * sizeof(int));
  for (int lv = 0; lv < N->nlev && rc == ORC_OK; lv++) {
    int a = N->lptr[lv], b = N->lptr[lv + 1];
    int nbig = 0;   /* fronts are sorted largest first */
    while (a + nbig < b && front_work(S, N->lfront[a + nbig]) > big) nbig++;
    for (int q = a; q < a + nbig && rc == ORC_OK; q++) rc = factor_one(N, N->lfront[q], hdiag, hoff, lam, rel0);
    int bad = 0;
#pragma omp parallel if (b - a - nbig > 1)
    {
      int *rel = (int *)malloc((S->n > 0 ? S->n : 1) * sizeof(int));
#pragma omp for schedule(dynamic, 1)
      for (int q = a + nbig; q < b; q++)
        if (factor_one(N, N->lfront[q], hdiag, hoff, lam, rel) != ORC_OK) {
#pragma omp atomic write
          bad = 1;
        }
      free(rel);
    }
    if (bad) rc = ORC_E_INDETERMINANT;
  }
  free(rel0);
  for (int s = 0; s < S->ns; s++) { /* a failed factorisation leaves updates behind */
    free(N->U[s]);
    N->U[s] = NULL;
  }
  return rc;
}

/* x (old pose order, 3 per pose) <- (L L^T)^-1 b */
static void num_solve(chol_num *N, const double *b, double *x) {
  chol_sym *S = N->S;
  int n = S->n;
  double *y = (double *)malloc((size_t)(3 * n > 0 ? 3 * n : 1) * sizeof(double));
  for (int k = 0; k < n; k++)
    for (int a = 0; a < 3; a++) y[3 * k + a] = b[3 * S->perm[k] + a];
  double *tmp = (double *)malloc((size_t)(S->maxfront > 0 ? S->maxfront : 1) * sizeof(double));
  /* forward: L y = b */
  for (int s = 0; s < S->ns; s++) {
    int f = S->sfirst[s], l = S->sfirst[s + 1];
    int nb = S->rptr[s + 1] - S->rptr[s];
    const int *R = S->rows + S->rptr[s];
    int m = 3 * (l - f + nb), wd = 3 * (l - f);
    const double *P = N->L + S->loff[s];
    double *ys = y + 3 * f;
    for (int j = 0; j < wd; j++) {
      ys[j] /= P[j + (size_t)j * m];
      double v = ys[j];
      for (int i = j + 1; i < wd; i++) ys[i] -= P[i + (size_t)j * m] * v;
    }
    int mb = m - wd;
    /* tmp = L21 y: a big front's rows spread over the threads (every element
     * summed over j in the same order) */
    const int nrb = (mb + 255) / 256;
#pragma omp parallel for schedule(static) if ((double)mb * wd > 1e6)
    for (int rb = 0; rb < nrb; rb++) {
      const int i0 = 256 * rb, i1 = i0 + 256 < mb ? i0 + 256 : mb;
      for (int i = i0; i < i1; i++) tmp[i] = 0;
      for (int j = 0; j < wd; j++) {
        double v = ys[j];
        const double *col = P + wd + (size_t)j * m;
        for (int i = i0; i < i1; i++) tmp[i] += col[i] * v;
      }
    }
    for (int t = 0; t < nb; t++)
      for (int a = 0; a < 3; a++) y[3 * R[t] + a] -= tmp[3 * t + a];
  }
  /* backward: L^T x = y */
  for (int s = S->ns - 1; s >= 0; s--) {
    int f = S->sfirst[s], l = S->sfirst[s + 1];
    int nb = S->rptr[s + 1] - S->rptr[s];
    const int *R = S->rows + S->rptr[s];
    int m = 3 * (l - f + nb), wd = 3 * (l - f);
    const double *P = N->L + S->loff[s];
    double *ys = y + 3 * f;
    int mb = m - wd;
    for (int t = 0; t < nb; t++)
      for (int a = 0; a < 3; a++) tmp[3 * t + a] = y[3 * R[t] + a];
#pragma omp parallel for schedule(static) if ((double)mb * wd > 1e6)
    for (int j = 0; j < wd; j++) {
      const double *col = P + wd + (size_t)j * m;
      double acc = 0;
      for (int i = 0; i < mb; i++) acc += col[i] * tmp[i];
      ys[j] -= acc;
    }
    for (int j = wd - 1; j >= 0; j--) {
      double v = ys[j];
      for (int i = j + 1; i < wd; i++) v -= P[i + (size_t)j * m] * ys[i];
      ys[j] = v / P[j + (size_t)j * m];
    }
  }
  for (int k = 0; k < n; k++)
    for (int a = 0; a < 3; a++) x[3 * S->perm[k] + a] = y[3 * k + a];
  free(y);
  free(tmp);
}

/* ------------------------------------------------------------- the problem */
typedef struct {
  int n, ne, np;
  int32_t *ei, *ej, *pi;
  pose2 *ez, *pz;
  double *eom, *pom; /* 9 each, row-major */
  chol_sym *S;
  chol_num *N;
  /* linearisation workspace */
  double *hdiag, *hoff, *g, *ee, *ep, *J1;
  double t_symbolic;
} orc;

void orc_default_params(orc_params *p) {
  p->max_iterations = 100;
  p->relative_error_tol = 1e-5;
  p->absolute_error_tol = 1e-5;
  p->error_tol = 0.0;
  p->lambda_initial = 1e-5;
  p->lambda_factor = 10.0;
  p->lambda_upper_bound = 1e5;
  p->lambda_lower_bound = 0.0;
  p->min_model_fidelity = 1e-3;
  p->use_fixed_lambda_factor = 1;
  p->algorithm = 0;
  p->max_outer = 0;
}

void orc_destroy(void *h) {
  orc *o = (orc *)h;
  if (!o) return;
  free(o->ei);
  free(o->ej);
  free(o->pi);
  free(o->ez);
  free(o->pz);
  free(o->eom);
  free(o->pom);
  num_free(o->N);   /* reads the symbolic sizes: before sym_free */
  sym_free(o->S);
  free(o->hdiag);
  free(o->hoff);
  free(o->g);
  free(o->ee);
  free(o->ep);
  free(o->J1);
  free(o);
}

void *orc_create_ordered(int n, int ne, const int32_t *ei, const int32_t *ej, const double *ez,
                         const double *ecov, int np, const int32_t *pi, const double *pz,
                         const double *pcov, const int32_t *order, int *status);

void *orc_create(int n, int ne, const int32_t *ei, const int32_t *ej, const double *ez,
                 const double *ecov, int np, const int32_t *pi, const double *pz,
                 const double *pcov, int *status) {
  return orc_create_ordered(n, ne, ei, ej, ez, ecov, np, pi, pz, pcov, NULL, status);
}

/* OpenMP threads of the factorisation / linearisation (bench.py times 1 and all) */
void orc_set_threads(int t) {
  if (t > 0) omp_set_num_threads(t);
}

void *orc_create_ordered(int n, int ne, const int32_t *ei, const int32_t *ej, const double *ez,
                         const double *ecov, int np, const int32_t *pi, const double *pz,
                         const double *pcov, const int32_t *order, int *status) {
  *status = ORC_OK;
  if (n < 0 || ne < 0 || np < 0) {
    *status = ORC_E_ARG;
    return NULL;
  }
  orc *o = (orc *)calloc(1, sizeof(orc));
  o->n = n;
  o->ne = ne;
  o->np = np;
  size_t E = ne > 0 ? ne : 1, P = np > 0 ? np : 1, Nn = n > 0 ? n : 1;
  o->ei = (int32_t *)malloc(E * 4);
  o->ej = (int32_t *)malloc(E * 4);
  o->pi = (int32_t *)malloc(P * 4);
  o->ez = (pose2 *)malloc(E * sizeof(pose2));
  o->pz = (pose2 *)malloc(P * sizeof(pose2));
  o->eom = (double *)malloc(E * 9 * 8);
  o->pom = (double *)malloc(P * 9 * 8);
  for (int e = 0; e < ne; e++) {
    if (ei[e] < 0 || ei[e] >= n || ej[e] < 0 || ej[e] >= n || ei[e] == ej[e]) {
      *status = ORC_E_ARG;
      orc_destroy(o);
      return NULL;
    }
    o->ei[e] = ei[e];
    o->ej[e] = ej[e];
    o->ez[e] = pose_from_xyt(ez + 3 * (size_t)e);
    if (orc_information(ecov + 9 * (size_t)e, o->eom + 9 * (size_t)e) != ORC_OK) {
      *status = ORC_E_BAD_COV;
      orc_destroy(o);
      return NULL;
    }
  }
  for (int k = 0; k < np; k++) {
    if (pi[k] < 0 || pi[k] >= n) {
      *status = ORC_E_ARG;
      orc_destroy(o);
      return NULL;
    }
    o->pi[k] = pi[k];
    o->pz[k] = pose_from_xyt(pz + 3 * (size_t)k);
    if (orc_information(pcov + 9 * (size_t)k, o->pom + 9 * (size_t)k) != ORC_OK) {
      *status = ORC_E_BAD_COV;
      orc_destroy(o);
      return NULL;
    }
  }
  double t0 = now_s();
  if (order) { /* must be a permutation of 0..n-1 */
    char *seen = (char *)calloc(Nn, 1);
    int ok = 1;
    for (int k = 0; k < n && ok; k++) {
      if (order[k] < 0 || order[k] >= n || seen[order[k]]) ok = 0;
      else seen[order[k]] = 1;
    }
    free(seen);
    if (!ok) {
      *status = ORC_E_ARG;
      orc_destroy(o);
      return NULL;
    }
  }
  o->S = sym_analyze(n, ne, o->ei, o->ej, order);
  o->N = num_create(o->S);
  o->t_symbolic = now_s() - t0;
  o->hdiag = (double *)malloc(Nn * 9 * 8);
  o->hoff = (double *)malloc(E * 9 * 8);
  o->g = (double *)malloc(Nn * 3 * 8);
  o->ee = (double *)malloc(E * 3 * 8);
  o->ep = (double *)malloc(P * 3 * 8);
  o->J1 = (double *)malloc(E * 9 * 8);
  return o;
}

static inline double quad3(const double *om, const double *e) {
  double s = 0;
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) s += e[a] * om[3 * a + b] * e[b];
  return s;
}

static double graph_error(const orc *o, const pose2 *P) {
  double err = 0;
#pragma omp parallel for reduction(+ : err) schedule(static) if (o->ne > 20000)
  for (int e = 0; e < o->ne; e++) {
    double r[3];
    local3(o->ez[e], between(P[o->ei[e]], P[o->ej[e]]), r);
    err += 0.5 * quad3(o->eom + 9 * (size_t)e, r);
  }
  for (int k = 0; k < o->np; k++) {
    double r[3];
    local3(P[o->pi[k]], o->pz[k], r);
    r[0] = -r[0];
    r[1] = -r[1];
    r[2] = -r[2];
    err += 0.5 * quad3(o->pom + 9 * (size_t)k, r);
  }
  return err;
}

/* NonlinearFactorGraph::linearize + the Hessian blocks the elimination forms */
static double linearize(orc *o, const pose2 *P) {
  int n = o->n;
  memset(o->hdiag, 0, (size_t)n * 9 * 8);
  memset(o->g, 0, (size_t)n * 3 * 8);
  double err = 0;
#pragma omp parallel for reduction(+ : err) schedule(static) if (o->ne > 20000)
  for (int e = 0; e < o->ne; e++) {
    pose2 p1 = P[o->ei[e]], p2 = P[o->ej[e]];
    pose2 hx = between(p1, p2);
    double *r = o->ee + 3 * (size_t)e;
    local3(o->ez[e], hx, r);
    double x = p2.x - p1.x, y = p2.y - p1.y;
    double *J = o->J1 + 9 * (size_t)e;
    J[0] = -hx.c; J[1] = -hx.s; J[2] = -p2.s * x + p2.c * y;
    J[3] = hx.s;  J[4] = -hx.c; J[5] = -p2.c * x - p2.s * y;
    J[6] = 0.0;   J[7] = 0.0;   J[8] = -1.0;
    const double *om = o->eom + 9 * (size_t)e;
    double *B = o->hoff + 9 * (size_t)e; /* J1^T Omega */
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += J[3 * k + a] * om[3 * k + b];
        B[3 * a + b] = s;
      }
    err += 0.5 * quad3(om, r);
  }
  /* accumulate per pose (serial: deterministic order) */
  for (int e = 0; e < o->ne; e++) {
    const double *B = o->hoff + 9 * (size_t)e, *J = o->J1 + 9 * (size_t)e;
    const double *om = o->eom + 9 * (size_t)e, *r = o->ee + 3 * (size_t)e;
    double *Di = o->hdiag + 9 * (size_t)o->ei[e], *Dj = o->hdiag + 9 * (size_t)o->ej[e];
    double *gi = o->g + 3 * (size_t)o->ei[e], *gj = o->g + 3 * (size_t)o->ej[e];
    for (int a = 0; a < 3; a++) {
      for (int b = 0; b < 3; b++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += B[3 * a + k] * J[3 * k + b];
        Di[3 * a + b] += s;
        Dj[3 * a + b] += om[3 * a + b];
      }
      gi[a] += B[3 * a] * r[0] + B[3 * a + 1] * r[1] + B[3 * a + 2] * r[2];
      gj[a] += om[3 * a] * r[0] + om[3 * a + 1] * r[1] + om[3 * a + 2] * r[2];
    }
  }
  for (int k = 0; k < o->np; k++) {
    double *r = o->ep + 3 * (size_t)k;
    local3(P[o->pi[k]], o->pz[k], r);
    r[0] = -r[0];
    r[1] = -r[1];
    r[2] = -r[2];
    const double *om = o->pom + 9 * (size_t)k;
    double *D = o->hdiag + 9 * (size_t)o->pi[k], *gp = o->g + 3 * (size_t)o->pi[k];
    for (int a = 0; a < 9; a++) D[a] += om[a];
    for (int a = 0; a < 3; a++) gp[a] += om[3 * a] * r[0] + om[3 * a + 1] * r[1] + om[3 * a + 2] * r[2];
    err += 0.5 * quad3(om, r);
  }
  return err;
}

/* GaussianFactorGraph::error(delta) = 0.5 sum |R (J delta + e)|^2 */
static double linear_error(const orc *o, const double *d) {
  double err = 0;
#pragma omp parallel for reduction(+ : err) schedule(static) if (o->ne > 20000)
  for (int e = 0; e < o->ne; e++) {
    const double *J = o->J1 + 9 * (size_t)e, *r = o->ee + 3 * (size_t)e;
    const double *di = d ? d + 3 * (size_t)o->ei[e] : NULL, *dj = d ? d + 3 * (size_t)o->ej[e] : NULL;
    double v[3];
    for (int a = 0; a < 3; a++) {
      v[a] = r[a];
      if (d) v[a] += J[3 * a] * di[0] + J[3 * a + 1] * di[1] + J[3 * a + 2] * di[2] + dj[a];
    }
    err += 0.5 * quad3(o->eom + 9 * (size_t)e, v);
  }
  for (int k = 0; k < o->np; k++) {
    const double *r = o->ep + 3 * (size_t)k;
    double v[3];
    for (int a = 0; a < 3; a++) v[a] = r[a] + (d ? d[3 * (size_t)o->pi[k] + a] : 0.0);
    err += 0.5 * quad3(o->pom + 9 * (size_t)k, v);
  }
  return err;
}

static int solve_damped(orc *o, double lam, double *delta, double *tf, double *ts) {
  double t0 = now_s();
  int rc = num_factor(o->N, o->hdiag, o->hoff, lam);
  double t1 = now_s();
  *tf += t1 - t0;
  if (rc) return rc;
  double *rhs = (double *)malloc((size_t)(3 * o->n > 0 ? 3 * o->n : 1) * 8);
  for (int i = 0; i < 3 * o->n; i++) rhs[i] = -o->g[i];
  num_solve(o->N, rhs, delta);
  free(rhs);
  *ts += now_s() - t1;
  for (int i = 0; i < 3 * o->n; i++)
    if (!isfinite(delta[i])) return ORC_E_INDETERMINANT;
  return ORC_OK;
}

static int check_convergence(const orc_params *p, double cur, double nw) {
  if (nw <= p->error_tol) return 1;
  double absd = cur - nw;
  double reld = absd / cur;
  return (p->relative_error_tol != 0.0 && reld <= p->relative_error_tol) || absd <= p->absolute_error_tol;
}

int orc_optimize(void *h, const double *init, const orc_params *prm, double *out, orc_stats *st,
                 double *trace, int trace_cap, int *trace_len) {
  orc *o = (orc *)h;
  orc_params dp;
  if (!prm) {
    orc_default_params(&dp);
    prm = &dp;
  }
  orc_stats S;
  memset(&S, 0, sizeof(S));
  int ntr = 0;
  double T0 = now_s();
  int n = o->n;
  size_t Nn = n > 0 ? n : 1;
  pose2 *P = (pose2 *)malloc(Nn * sizeof(pose2)), *C = (pose2 *)malloc(Nn * sizeof(pose2));
  double *delta = (double *)malloc(Nn * 3 * 8);
  for (int k = 0; k < n; k++) P[k] = pose_from_xyt(init + 3 * (size_t)k);
  double t = now_s();
  double err = graph_error(o, P);
  S.t_error += now_s() - t;
  S.initial_error = err;
  double lam = prm->lambda_initial, factor = prm->lambda_factor;
  int iters = 0, inner = 0, rc = ORC_OK;
  S.factor_flops = o->S->flops;
  S.nnz_l = o->S->nnzl;
  S.nsuper = o->S->ns;
  S.t_symbolic = o->t_symbolic;
  if (!(err <= prm->error_tol) && iters < prm->max_iterations) {
    double new_err = err;
    for (;;) {
      double cur_err = new_err;
      t = now_s();
      linearize(o, P);
      S.t_linearize += now_s() - t;
      S.linearizations++;
      if (prm->algorithm == 1) { /* Gauss-Newton */
        rc = solve_damped(o, 0.0, delta, &S.t_factor, &S.t_solve);
        if (rc) break;
        for (int k = 0; k < n; k++) P[k] = retract(P[k], delta + 3 * (size_t)k);
        t = now_s();
        err = graph_error(o, P);
        S.t_error += now_s() - t;
        iters++;
        inner++;
        if (trace && ntr < trace_cap) {
          double *tr = trace + 7 * (size_t)ntr++;
          tr[0] = iters; tr[1] = 0; tr[2] = 1; tr[3] = NAN; tr[4] = err; tr[5] = 0; tr[6] = 1;
        }
      } else {
        for (;;) { /* tryLambda */
          double fidelity = 0.0, new_e = INFINITY, lin_change = NAN;
          int success = 0, stop = 0;
          int solved = solve_damped(o, lam, delta, &S.t_factor, &S.t_solve) == ORC_OK;
          if (solved) {
            double old_lin = linear_error(o, NULL);
            double new_lin = linear_error(o, delta);
            lin_change = old_lin - new_lin;
            if (lin_change >= 0) {
              for (int k = 0; k < n; k++) C[k] = retract(P[k], delta + 3 * (size_t)k);
              t = now_s();
              new_e = graph_error(o, C);
              S.t_error += now_s() - t;
              double cost_change = err - new_e;
              if (lin_change > 2.220446049250313e-16 * old_lin) {
                fidelity = cost_change / lin_change;
                success = fidelity > prm->min_model_fidelity;
              }
              if (fabs(cost_change) < prm->relative_error_tol * err) stop = 1;
            }
          }
          if (trace && ntr < trace_cap) {
            double *tr = trace + 7 * (size_t)ntr++;
            tr[0] = iters; tr[1] = lam; tr[2] = solved; tr[3] = lin_change;
            tr[4] = new_e; tr[5] = fidelity; tr[6] = success;
          }
          if (success) {
            if (prm->use_fixed_lambda_factor) lam /= prm->lambda_factor;
            else {
              double q = 2.0 * fidelity - 1.0;
              double f = 1.0 - q * q * q;
              lam *= f > 1.0 / 3.0 ? f : 1.0 / 3.0;
              factor *= 2.0;
            }
            if (lam < prm->lambda_lower_bound) lam = prm->lambda_lower_bound;
            pose2 *tmp = P;
            P = C;
            C = tmp;
            err = new_e;
            iters++;
            inner++;
            break;
          }
          if (!stop) {
            lam *= factor;
            inner++;
            if (!prm->use_fixed_lambda_factor) factor *= 2.0;
            if (lam >= prm->lambda_upper_bound) break;
            continue;
          }
          break;
        }
      }
      new_err = err;
      if (prm->max_outer > 0 && S.linearizations >= prm->max_outer) break;
      if (!(iters < prm->max_iterations && !check_convergence(prm, cur_err, new_err) && isfinite(cur_err)))
        break;
    }
  }
  for (int k = 0; k < n; k++) {
    out[3 * k] = P[k].x;
    out[3 * k + 1] = P[k].y;
    out[3 * k + 2] = atan2(P[k].s, P[k].c);
  }
  S.iterations = iters;
  S.inner_iterations = inner;
  S.final_error = err;
  S.status = rc;
  S.t_total = now_s() - T0;
  if (st) *st = S;
  if (trace_len) *trace_len = ntr;
  free(P);
  free(C);
  free(delta);
  return rc;
}

int orc_linearize(void *h, const double *poses, double *hdiag, double *hoff, double *g, double *err) {
  orc *o = (orc *)h;
  size_t Nn = o->n > 0 ? o->n : 1;
  pose2 *P = (pose2 *)malloc(Nn * sizeof(pose2));
  for (int k = 0; k < o->n; k++) P[k] = pose_from_xyt(poses + 3 * (size_t)k);
  double e = linearize(o, P);
  if (hdiag) memcpy(hdiag, o->hdiag, (size_t)o->n * 9 * 8);
  if (hoff) memcpy(hoff, o->hoff, (size_t)o->ne * 9 * 8);
  if (g) memcpy(g, o->g, (size_t)o->n * 3 * 8);
  if (err) *err = e;
  free(P);
  return ORC_OK;
}

int orc_solve(void *h, const double *poses, double lambda, double *delta) {
  orc *o = (orc *)h;
  size_t Nn = o->n > 0 ? o->n : 1;
  pose2 *P = (pose2 *)malloc(Nn * sizeof(pose2));
  for (int k = 0; k < o->n; k++) P[k] = pose_from_xyt(poses + 3 * (size_t)k);
  linearize(o, P);
  double tf = 0, ts = 0;
  int rc = solve_damped(o, lambda, delta, &tf, &ts);
  free(P);
  return rc;
}

int orc_supernodes(void *h, int *m, int *w, int *parent) {
  orc *o = (orc *)h;
  chol_sym *S = o->S;
  if (m)
    for (int s = 0; s < S->ns; s++) {
      int wp = S->sfirst[s + 1] - S->sfirst[s];
      m[s] = 3 * (wp + S->rptr[s + 1] - S->rptr[s]);
      w[s] = 3 * wp;
      parent[s] = S->sparent[s];
    }
  return S->ns;
}

double orc_error(void *h, const double *poses) {
  orc *o = (orc *)h;
  size_t Nn = o->n > 0 ? o->n : 1;
  pose2 *P = (pose2 *)malloc(Nn * sizeof(pose2));
  for (int k = 0; k < o->n; k++) P[k] = pose_from_xyt(poses + 3 * (size_t)k);
  double e = graph_error(o, P);
  free(P);
  return e;
}

/* ---- closest_keyframe service ----------------------------
 * Restates /root/reference/src/graph/src/graph.cpp:146-178: with
 * keyframes.size() > keyframes_to_skip_in_loop_closing (graph.cpp:15, = 10),
 * distances to keyframes[0 .. size - skip - 1] are
 * sqrt(pow(x2 - x1, 2) + pow(y2 - y1, 2)) (:153-158), and the first index with
 * the smallest distance wins (strict <, :161-166).  Returns the index or -1
 * when there are not enough keyframes (:170-171, service returns false).
 * fp-contract off: the reference's x86-64 build has no FMA contraction. */
__attribute__((optimize("fp-contract=off")))
int orc_closest_keyframe(int n, const double *xy, double qx, double qy, int skip, double *dist) {
  if (n <= 0 || n <= skip) return -1;
  int best = 0;
  double dbest = 0.0;
  for (int i = 0; i < n - skip; i++) {
    const double d = sqrt(pow(xy[2 * i] - qx, 2) + pow(xy[2 * i + 1] - qy, 2));
    if (i == 0 || d < dbest) {
      best = i;
      dbest = d;
    }
  }
  *dist = dbest;
  return best;
}
