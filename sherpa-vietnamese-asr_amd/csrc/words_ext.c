/* _zasr_words: the decode_chunk word post-processing (core/asr_engine.py:1227-1326: BPE
 * pieces -> word dicts with timestamps, probabilities and the entropy aggregates of
 * :1159-1206) as a CPython extension.  Same arithmetic as the Python restatement
 * zasr.asr_engine._words_from_search, operation for operation in IEEE double:
 *   - Python's round(x, 4) is the correctly rounded 4-decimal value of x read back as a
 *     double; glibc's "%.4f" + strtod compute the same (no binary double lies exactly half
 *     way between two 4-decimal values, so the tie rule never applies);
 *   - math.exp / math.log / ** are libm's exp / log / pow (the same libm in this process);
 *   - sum(list) is a left-to-right double sum; np.mean of a Python float list is numpy's
 *     float64 pairwise sum (numpy/_core/src/umath/loops_utils.h.src) divided by the count.
 * The dict keys are inserted in the Python version's order, so the dicts compare and
 * serialise identically.  tests/test_words_ext.py checks both against each other. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

/* Python's round(x, 4): the double nearest to the 4-decimal value d / 10^4 nearest to x.
   d from the exact product x * 10^4 = p + err (err by FMA, exact): floor(p) or floor(p) + 1
   by the sign of (p - floor(p) - 0.5) + err, decided exactly (no binary double sits on a tie,
   see above; an exact tie would take the even d like Python).  d / 10000.0 is then one
   correctly rounded division -- what strtod returns for the decimal string.  Values too
   large for an exact d take the snprintf / strtod route. */
static double round4_slow(double x) {
  char buf[400];
  snprintf(buf, sizeof buf, "%.4f", x);
  return strtod(buf, NULL);
}

static double round4(double x) {
  if (!isfinite(x)) return x;
  const double ax = fabs(x);
  if (ax >= 4.0e11) return round4_slow(x);
  const double p = ax * 10000.0;
  const double err = fma(ax, 10000.0, -p);  /* ax * 10^4 = p + err exactly */
  const double fl = floor(p);
  const double frac = p - fl;               /* exact */
  const double t = frac - 0.5;              /* exact: frac in [0, 1) with p's ulp, |t| <= 0.5 */
  double d = fl;
  if (t > -err) d = fl + 1.0;               /* frac + err > 0.5 */
  else if (t == -err && fmod(fl, 2.0) != 0.0) d = fl + 1.0;
  if (frac == 0.0 && err < 0.0) d = fl;     /* (p + err) just below an integer: floor is fl - 1,
                                               but then frac + 1 + err > 0.5 gives fl */
  const double r = d / 10000.0;
  return copysign(r, x);
}

/* numpy float64 pairwise sum */
static double pairwise(const double* a, Py_ssize_t n) {
  if (n < 8) {
    double res = -0.0;
    for (Py_ssize_t i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    Py_ssize_t i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  Py_ssize_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise(a, n2) + pairwise(a + n2, n - n2);
}

typedef struct {
  double tsallis_norm, margin, entropy_norm;
} Ent;

/* dict keys, interned once (PyDict_SetItemString would build and intern a str per call) */
enum { K_TEXT, K_START, K_END, K_LSTART, K_LEND, K_PROB, K_TSMAX, K_MMIN, K_ENORM, K_CONF, K_TOKS,
       K_TSL, K_N };
static const char* const kKeyNames[K_N] = {
    "text", "start", "end", "local_start", "local_end", "prob", "tsallis_max", "margin_min",
    "entropy_norm", "_conf", "_chunk_bpe_tokens", "_chunk_bpe_timestamps_local"};
static PyObject* kKeys[K_N];

static int set_f(PyObject* d, int key, double v) {
  PyObject* o = PyFloat_FromDouble(v);
  if (!o) return -1;
  int rc = PyDict_SetItem(d, kKeys[key], o);
  Py_DECREF(o);
  return rc;
}

/* _finalize_word_entropy (:1187-1206) of one word: probs / ents of its pieces */
static int finalize(PyObject* w, const double* probs, Py_ssize_t np_, const Ent* ents,
                    Py_ssize_t ne, double* scratch) {
  double s = 0.0;
  for (Py_ssize_t i = 0; i < np_; ++i) s += probs[i];
  if (set_f(w, K_PROB, s / (double)np_) < 0) return -1;
  if (ne == 0) {
    for (int i = K_TSMAX; i <= K_CONF; ++i)
      if (PyDict_SetItem(w, kKeys[i], Py_None) < 0) return -1;
    return 0;
  }
  double tmax = ents[0].tsallis_norm, mmin = ents[0].margin, conf = 0.0;
  for (Py_ssize_t i = 0; i < ne; ++i) {
    if (ents[i].tsallis_norm > tmax) tmax = ents[i].tsallis_norm;
    if (ents[i].margin < mmin) mmin = ents[i].margin;
    scratch[i] = ents[i].entropy_norm;
    conf += ents[i].margin * (1.0 - ents[i].tsallis_norm);
  }
  if (set_f(w, K_TSMAX, round4(tmax)) < 0) return -1;
  if (set_f(w, K_MMIN, round4(mmin)) < 0) return -1;
  if (set_f(w, K_ENORM, round4(pairwise(scratch, ne) / (double)ne)) < 0) return -1;
  if (set_f(w, K_CONF, round4(conf / (double)ne)) < 0) return -1;
  return 0;
}

/* text.startswith(" ") or text.startswith("▁") */
static int starts_word(PyObject* text) {
  if (PyUnicode_GET_LENGTH(text) == 0) return 0;
  const Py_UCS4 c = PyUnicode_READ_CHAR(text, 0);
  return c == 0x20 || c == 0x2581;
}

/* text.lstrip(" ").lstrip("▁") (a new reference) */
static PyObject* strip_word_start(PyObject* text) {
  const Py_ssize_t n = PyUnicode_GET_LENGTH(text);
  Py_ssize_t i = 0;
  while (i < n && PyUnicode_READ_CHAR(text, i) == 0x20) ++i;
  while (i < n && PyUnicode_READ_CHAR(text, i) == 0x2581) ++i;
  return PyUnicode_Substring(text, i, n);
}

static int get_buf(PyObject* o, Py_buffer* b, Py_ssize_t itemsize, const char* what) {
  if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS) < 0) return -1;
  if (b->itemsize != itemsize && b->len > 0) {
    PyErr_Format(PyExc_TypeError, "%s: expected %zd-byte elements", what, itemsize);
    PyBuffer_Release(b);
    return -1;
  }
  return 0;
}

/* words_from_search(pieces, lowered, V, n_samples, time_offset, token_ids int32,
 *                   frames int32, log_probs float64, T, stats float32 [k][4])
 * pieces / lowered: per token id, the token string and its .lower() (lists of length V'; ids
 * outside map to "", as id2token.get(t, "")). */
static PyObject* words_from_search(PyObject* self, PyObject* args) {
  PyObject *pieces, *lowered, *o_tok, *o_fr, *o_lp, *o_st;
  long V, n_samples, T;
  double time_offset;
  if (!PyArg_ParseTuple(args, "O!O!lldOOOlO", &PyList_Type, &pieces, &PyList_Type, &lowered, &V,
                        &n_samples, &time_offset, &o_tok, &o_fr, &o_lp, &T, &o_st))
    return NULL;
  /* the two tables are indexed with the same bounds check: equal lengths, str entries */
  if (PyList_GET_SIZE(lowered) != PyList_GET_SIZE(pieces)) {
    PyErr_SetString(PyExc_ValueError, "words_from_search: pieces and lowered differ in length");
    return NULL;
  }
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(pieces); ++i) {
    if (!PyUnicode_Check(PyList_GET_ITEM(pieces, i)) || !PyUnicode_Check(PyList_GET_ITEM(lowered, i))) {
      PyErr_SetString(PyExc_TypeError, "words_from_search: vocabulary entries must be str");
      return NULL;
    }
  }
  Py_buffer bt, bf, bl, bs;
  if (get_buf(o_tok, &bt, 4, "token_ids") < 0) return NULL;
  if (get_buf(o_fr, &bf, 4, "frames") < 0) { PyBuffer_Release(&bt); return NULL; }
  if (get_buf(o_lp, &bl, 8, "log_probs") < 0) { PyBuffer_Release(&bt); PyBuffer_Release(&bf); return NULL; }
  if (get_buf(o_st, &bs, 4, "stats") < 0) {
    PyBuffer_Release(&bt); PyBuffer_Release(&bf); PyBuffer_Release(&bl);
    return NULL;
  }
  PyObject* words = PyList_New(0);
  double *ts = NULL, *probs = NULL, *scratch = NULL;
  Ent* ents = NULL;
  PyObject* cur = NULL;
  const Py_ssize_t k = bt.len / 4;
  const Py_ssize_t nfr = bf.len / 4, nlp = bl.len / 8, nst = bs.len / 16;
  const Py_ssize_t ntab = PyList_GET_SIZE(pieces);
  const int* tok = (const int*)bt.buf;
  const int* fr = (const int*)bf.buf;
  const double* lp = (const double*)bl.buf;
  const float* st = (const float*)bs.buf;
  PyObject* empty = PyUnicode_FromString("");
  Py_ssize_t* wst = NULL;
  if (!words || !empty) goto fail;
  if (k == 0 || T <= 0 || nfr < k) goto done;
  ts = (double*)malloc(sizeof(double) * k);
  probs = (double*)malloc(sizeof(double) * k);
  scratch = (double*)malloc(sizeof(double) * k);
  ents = (Ent*)malloc(sizeof(Ent) * k);
  wst = (Py_ssize_t*)malloc(sizeof(Py_ssize_t) * (k + 1));
  if (!ts || !probs || !scratch || !ents || !wst) { PyErr_NoMemory(); goto fail; }
  {
    const double chunk_dur = (double)n_samples / 16000.0;
    for (Py_ssize_t j = 0; j < k; ++j) ts[j] = (double)fr[j] / (double)T * chunk_dur;
    const double avg = k >= 2 ? (ts[k - 1] - ts[0]) / (double)(k - 1) : 0.08;
    /* _compute_token_entropy (:1159-1181) */
    const double alpha = 1.0 / 3.0;
    const double max_entropy = V > 1 ? log((double)V) : 1.0;
    const double ts_max = V > 1 ? (1.0 / (alpha - 1.0)) * (1.0 - pow((double)V, 1.0 - alpha)) : 1.0;
    for (Py_ssize_t j = 0; j < k; ++j) {
      if (j < nst) {
        const double entropy = st[4 * j], s3 = st[4 * j + 1], top1 = st[4 * j + 2], top2 = st[4 * j + 3];
        const double tsallis = (1.0 / (alpha - 1.0)) * (1.0 - s3);
        ents[j].tsallis_norm = round4(ts_max > 0 ? tsallis / ts_max : 0.0);
        ents[j].margin = round4(top1 - top2);
        ents[j].entropy_norm = round4(entropy / max_entropy);
      } else {
        ents[j].tsallis_norm = 0.0;
        ents[j].margin = 1.0;
        ents[j].entropy_norm = 0.0;
      }
      probs[j] = j < nlp ? exp(lp[j]) : 1.0;
    }
    /* word boundaries: a piece starting with " " or "▁" opens a word (:1227-1290) */
    Py_ssize_t nw = 0;
    for (Py_ssize_t j = 0; j < k; ++j) {
      const int id = tok[j];
      PyObject* text = (id >= 0 && id < ntab) ? PyList_GET_ITEM(lowered, id) : empty;
      if (j == 0 || starts_word(text)) wst[nw++] = j;
    }
    wst[nw] = k;
    /* one dict per word, keys in the order the reference's dicts end up with: text, start,
     * end, local_start, local_end (end: the last piece's start + the mean piece spacing, capped
     * at the next word's start, :1316-1322), then the entropy fields */
    for (Py_ssize_t i = 0; i < nw; ++i) {
      const Py_ssize_t a = wst[i], b = wst[i + 1];
      PyObject* first = (tok[a] >= 0 && tok[a] < ntab) ? PyList_GET_ITEM(lowered, tok[a]) : empty;
      PyObject* t = starts_word(first) ? strip_word_start(first) : (Py_INCREF(first), first);
      if (!t) goto fail;
      for (Py_ssize_t j = a + 1; j < b && t; ++j) {  /* cur["text"] += text */
        PyObject* x = (tok[j] >= 0 && tok[j] < ntab) ? PyList_GET_ITEM(lowered, tok[j]) : empty;
        PyObject* u = PyUnicode_Concat(t, x);
        Py_DECREF(t);
        t = u;
      }
      if (!t) goto fail;
      cur = PyDict_New();
      if (!cur) { Py_DECREF(t); goto fail; }
      int rc = PyDict_SetItem(cur, kKeys[K_TEXT], t);
      Py_DECREF(t);
      double end = (ts[b - 1] + time_offset) + avg;
      if (i + 1 < nw) {
        const double nxt = ts[b] + time_offset;
        if (nxt < end) end = nxt;  /* min(end, next start): the first argument on ties */
      }
      if (rc < 0 || set_f(cur, K_START, ts[a] + time_offset) < 0 || set_f(cur, K_END, end) < 0 ||
          set_f(cur, K_LSTART, ts[a]) < 0 || set_f(cur, K_LEND, end - time_offset) < 0 ||
          finalize(cur, probs + a, b - a, ents + a, b - a, scratch) < 0)
        goto fail;
      if (PyList_Append(words, cur) < 0) goto fail;
      Py_CLEAR(cur);
    }
    if (nw > 0) {
      PyObject* w = PyList_GET_ITEM(words, 0);
      PyObject* pl = PyList_New(k);
      PyObject* tl = PyList_New(k);
      if (!pl || !tl) { Py_XDECREF(pl); Py_XDECREF(tl); goto fail; }
      for (Py_ssize_t j = 0; j < k; ++j) {
        const int id = tok[j];
        PyObject* p = (id >= 0 && id < ntab) ? PyList_GET_ITEM(pieces, id) : empty;
        Py_INCREF(p);
        PyList_SET_ITEM(pl, j, p);
        PyObject* f = PyFloat_FromDouble(ts[j]);
        if (!f) { Py_DECREF(pl); Py_DECREF(tl); goto fail; }
        PyList_SET_ITEM(tl, j, f);
      }
      int rc = PyDict_SetItem(w, kKeys[K_TOKS], pl);
      Py_DECREF(pl);
      if (rc == 0) rc = PyDict_SetItem(w, kKeys[K_TSL], tl);
      Py_DECREF(tl);
      if (rc < 0) goto fail;
    }
  }
done:
  free(ts); free(probs); free(scratch); free(ents); free(wst);
  Py_XDECREF(empty);
  PyBuffer_Release(&bt); PyBuffer_Release(&bf); PyBuffer_Release(&bl); PyBuffer_Release(&bs);
  return words;
fail:
  Py_XDECREF(cur);
  Py_XDECREF(words);
  words = NULL;
  goto done;
}

static PyObject* py_round4(PyObject* self, PyObject* arg) {
  const double x = PyFloat_AsDouble(arg);
  if (x == -1.0 && PyErr_Occurred()) return NULL;
  return PyFloat_FromDouble(round4(x));
}

static PyMethodDef methods[] = {
    {"round4", py_round4, METH_O, "round(x, 4) as the word builder computes it (tests)"},
    {"words_from_search", words_from_search, METH_VARARGS,
     "decode_chunk's BPE -> word dicts (core/asr_engine.py:1227-1326)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_zasr_words", NULL, -1, methods};

PyMODINIT_FUNC PyInit__zasr_words(void) {
  for (int i = 0; i < K_N; ++i)
    if (!kKeys[i] && !(kKeys[i] = PyUnicode_InternFromString(kKeyNames[i]))) return NULL;
  return PyModule_Create(&module);
}
