// hostpack.cpp -- plenum_amd._hostpack: the host half of the authenticator's
// batch path in native code (CPython extension, host CPU only).
//
// The reference does this per request in Python (plenum/server/client_authn.py:
// 89 b58decode(signature), :92 serializeForSig -> common/serializers/
// signing_serializer.py:35-91, nacl_wrappers.py:108 sig || msg).  SURVEY §8(f)
// row 2: with the verify on the GPU this host work is the bottleneck of the
// drop-in.  Every function here either returns the exact bytes the reference
// code produces or returns None ("take the Python path"), so the reference's
// exceptions (class, args, __cause__) are always raised by the Python
// restatement, never reimplemented here:
//   serialize_for_signing(obj, ignore) -> bytes | None
//       fast path for exact str / int / bool / float / None / list / dict with
//       str keys; float and int text come from PyObject_Str (Python's own repr),
//       key order from PyUnicode_Compare (list.sort on str).  Anything else
//       (subclasses, tuples, non-str keys, unencodable text) -> None.
//   b58decode(v) -> bytes | None        (base58 0.2.4 semantics; None on any
//                                        character outside the alphabet)
//   pack_split64(sigs, sers) -> (sig64, msgs, off, short)
//       crypto_sign_open's split of sm = sig || ser at byte 64, packed:
//       sig64 n*64 bytes, msgs + off (n+1 uint64 LE), short[i] = len(sm) < 64
//   pack_sm(sigs, sers, keys) -> (sm, off, pk32)   (edv_sign_open_batch layout)
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "host_pool.h"
#include <pthread.h>
#include <emmintrin.h>
#include <sched.h>
#include <unistd.h>
#include <sys/syscall.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <charconv>
#include <chrono>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

// ------------------------------------------------------------------ serialize

// The scan's serialization buffers: std::string's append is an out-of-line call per piece
// (a request's signing bytes are ~25 pieces); this one inlines to a bounds check + memcpy.
struct OutBuf {
  char* d = nullptr;
  size_t n = 0, cap = 0;
  OutBuf() = default;
  OutBuf(const OutBuf&) = delete;
  OutBuf& operator=(const OutBuf&) = delete;
  OutBuf(OutBuf&& o) noexcept : d(o.d), n(o.n), cap(o.cap) { o.d = nullptr, o.n = o.cap = 0; }
  ~OutBuf() { free(d); }
  size_t size() const { return n; }
  const char* data() const { return d; }
  void clear() { n = 0; }
  void reserve(size_t k) {
    if (k > cap) grow_to(k);
  }
  void resize(size_t k) {  // (shrinks only, in its callers)
    reserve(k);
    n = k;
  }
  void grow_to(size_t k) {
    const size_t c = std::max(k, cap * 2 + 256);
    char* q = (char*)realloc(d, c);
    if (!q) throw std::bad_alloc();
    d = q;
    cap = c;
  }
  void append(const char* src, size_t k) {
    if (n + k > cap) grow_to(n + k);
    copy_small(d + n, src, k);
    n += k;
  }
  // memcpy for the short pieces of a serialization (keys and values, mostly 1-64 bytes) inlined:
  // overlapping 16/8/4-byte moves, every load inside [src, src + k) and every store inside
  // [dst, dst + k) (libc's memcpy was an out-of-line call per piece)
  static inline void copy_small(char* dst, const char* src, size_t k) {
    if (k >= 16) {
      if (k > 64) {
        memcpy(dst, src, k);
        return;
      }
      for (size_t i = 0; i + 16 < k; i += 16)
        _mm_storeu_si128((__m128i*)(dst + i), _mm_loadu_si128((const __m128i*)(src + i)));
      _mm_storeu_si128((__m128i*)(dst + k - 16), _mm_loadu_si128((const __m128i*)(src + k - 16)));
    } else if (k >= 8) {
      uint64_t a, b;
      memcpy(&a, src, 8);
      memcpy(&b, src + k - 8, 8);
      memcpy(dst, &a, 8);
      memcpy(dst + k - 8, &b, 8);
    } else if (k >= 4) {
      uint32_t a, b;
      memcpy(&a, src, 4);
      memcpy(&b, src + k - 4, 4);
      memcpy(dst, &a, 4);
      memcpy(dst + k - 4, &b, 4);
    } else if (k) {
      dst[0] = src[0];
      dst[k / 2] = src[k / 2];
      dst[k - 1] = src[k - 1];
    }
  }
  void append(const char* z) { append(z, strlen(z)); }
  void append_short(const char* src, size_t k) {  // k <= 24 (a number's decimal text)
    if (n + k > cap) grow_to(n + k);
    memcpy(d + n, src, k < 24 ? k : 24);
    n += k;
  }
  void push_back(char c) {
    if (n + 1 > cap) grow_to(n + 1);
    d[n++] = c;
  }
};

template <class Out>
bool ser_obj(PyObject* o, int level, PyObject* ignore, Out& out);

inline void append_num(OutBuf& out, const char* b, size_t k) { out.append_short(b, k); }
inline void append_num(std::string& out, const char* b, size_t k) { out.append(b, k); }

template <class Out>
bool append_str(PyObject* s, Out& out) {
  if (PyUnicode_IS_ASCII(s)) {
    out.append((const char*)PyUnicode_1BYTE_DATA(s), (size_t)PyUnicode_GET_LENGTH(s));
    return true;
  }
  Py_ssize_t n = 0;
  const char* p = PyUnicode_AsUTF8AndSize(s, &n);
  if (!p) {
    PyErr_Clear();  // e.g. lone surrogates: the reference's encode raises -> Python path
    return false;
  }
  out.append(p, (size_t)n);
  return true;
}

template <class Out>
bool append_text_of(PyObject* o, Out& out) {  // str(o)
  PyObject* s = PyObject_Str(o);
  if (!s) {
    PyErr_Clear();
    return false;
  }
  const bool ok = append_str(s, out);
  Py_DECREF(s);
  return ok;
}

bool ignored(PyObject* k, PyObject* ignore) {
  if (!ignore) return false;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(ignore);
  PyObject** items = PySequence_Fast_ITEMS(ignore);
  for (Py_ssize_t i = 0; i < n; ++i) {
    if (PyUnicode_CheckExact(items[i]) && PyUnicode_Compare(k, items[i]) == 0) return true;
  }
  return false;
}

// str < str as list.sort orders them (code points); one-byte strings (the
// common case) compare with memcmp, others through PyUnicode_Compare.
bool str_less(PyObject* a, PyObject* b, bool& err) {
  if (PyUnicode_KIND(a) == PyUnicode_1BYTE_KIND && PyUnicode_KIND(b) == PyUnicode_1BYTE_KIND) {
    const Py_ssize_t na = PyUnicode_GET_LENGTH(a), nb = PyUnicode_GET_LENGTH(b);
    const int c = memcmp(PyUnicode_1BYTE_DATA(a), PyUnicode_1BYTE_DATA(b), (size_t)(na < nb ? na : nb));
    return c < 0 || (c == 0 && na < nb);
  }
  const int c = PyUnicode_Compare(a, b);
  if (c == -1 && PyErr_Occurred()) err = true;
  return c < 0;
}

template <class Out>
bool ser_dict(PyObject* d, int level, PyObject* ignore, Out& out) {
  // keys on the stack for ordinary dicts (insertion sort), a vector beyond
  constexpr Py_ssize_t kSmall = 24;
  PyObject* small[kSmall];
  std::vector<PyObject*> big;
  const Py_ssize_t nd = PyDict_GET_SIZE(d);
  PyObject** keys = small;
  if (nd > kSmall) {
    big.resize((size_t)nd);
    keys = big.data();
  }
  Py_ssize_t nk = 0, pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(d, &pos, &k, &v)) {
    if (!PyUnicode_CheckExact(k)) return false;  // non-str keys: the reference may raise -> Python path
    if (level == 0 && ignored(k, ignore)) continue;
    keys[nk++] = k;
  }
  bool cmp_err = false;
  if (nk <= kSmall) {
    for (Py_ssize_t i = 1; i < nk; ++i) {
      PyObject* x = keys[i];
      Py_ssize_t j = i;
      while (j > 0 && str_less(x, keys[j - 1], cmp_err)) {
        keys[j] = keys[j - 1];
        --j;
      }
      keys[j] = x;
    }
  } else {
    std::sort(keys, keys + nk, [&](PyObject* a, PyObject* b) { return str_less(a, b, cmp_err); });
  }
  if (cmp_err) {
    PyErr_Clear();
    return false;
  }
  for (Py_ssize_t i = 0; i < nk; ++i) {
    if (i) out.push_back('|');
    if (!append_str(keys[i], out)) return false;
    out.push_back(':');
    PyObject* val = PyDict_GetItem(d, keys[i]);  // borrowed
    if (!val || !ser_obj(val, level + 1, nullptr, out)) return false;
  }
  return true;
}

constexpr int kMaxDepth = 500;  // deeper: the Python path (which may hit RecursionError like the reference)

template <class Out>
bool ser_obj(PyObject* o, int level, PyObject* ignore, Out& out) {
  if (level > kMaxDepth) return false;
  if (PyUnicode_CheckExact(o)) return append_str(o, out);
  if (PyDict_CheckExact(o)) return ser_dict(o, level, ignore, out);
  if (PyList_CheckExact(o)) {
    const Py_ssize_t n = PyList_GET_SIZE(o);
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) out.push_back(',');
      if (!ser_obj(PyList_GET_ITEM(o, i), level + 1, nullptr, out)) return false;
    }
    return true;
  }
  if (o == Py_None) return true;
  if (PyBool_Check(o)) {
    out.append(o == Py_True ? "True" : "False");
    return true;
  }
  if (PyLong_CheckExact(o)) {  // str(int): decimal, without a temporary str for 64-bit values
    int overflow = 0;
    const long long x = PyLong_AsLongLongAndOverflow(o, &overflow);
    if (overflow || (x == -1 && PyErr_Occurred())) {
      PyErr_Clear();
      return append_text_of(o, out);
    }
    char b[24];
    const auto r = std::to_chars(b, b + sizeof b, x);  // str(int) for 64-bit values
    append_num(out, b, (size_t)(r.ptr - b));
    return true;
  }
  if (PyFloat_CheckExact(o)) return append_text_of(o, out);
  return false;  // tuples, sets, subclasses, other types: the Python path decides
}

PyObject* py_serialize_for_signing(PyObject*, PyObject* args) {
  PyObject *obj, *ignore = Py_None;
  if (!PyArg_ParseTuple(args, "O|O", &obj, &ignore)) return nullptr;
  PyObject* ign = nullptr;
  if (ignore != Py_None) {
    ign = PySequence_Fast(ignore, "ignore must be a sequence");
    if (!ign) return nullptr;
  }
  std::string out;
  out.reserve(256);
  const bool ok = ser_obj(obj, 0, ign, out);
  Py_XDECREF(ign);
  if (!ok) Py_RETURN_NONE;
  return PyBytes_FromStringAndSize(out.data(), (Py_ssize_t)out.size());
}

// ------------------------------------------------ serializer for worker threads
// scan_batch's worker threads serialize while the calling thread holds the GIL
// and waits for them: no Python code runs and no object changes meanwhile.
// The workers touch objects through pure reads only (exact-type checks,
// PyDict_Next, the data of one-byte strings, the digits of an exact int) -- no
// allocation, no reference counts, no error state (PyDict_GetItem would touch
// the GIL holder's error state, so the values come from PyDict_Next).  What
// needs more -- str() of a float or a big int, non-ASCII text, keys that are
// not one-byte strings -- is kDefer: ser_obj redoes that item under the GIL.
// kOk bytes equal ser_obj's; kFail exactly where ser_obj returns false.
enum WRes { kOk = 0, kFail = 1, kDefer = 2 };

WRes wser_obj(PyObject* o, int level, PyObject* ignore, OutBuf& out);

// A dict's key table read directly on CPython 3.10's combined-table layout
// (Objects/dict-common.h): the scan's workers walk a request's entries without a
// PyDict_Next call per key, and the prefetch pipeline walks ahead with it.  nullptr
// (and n = 0) for other layouts; elsewhere the workers use PyDict_Next.
#if PY_VERSION_HEX >= 0x030A0000 && PY_VERSION_HEX < 0x030B0000
struct DkEntry {
  Py_hash_t h;
  PyObject *k, *v;
};
struct DkHead {  // Objects/dict-common.h, 3.10
  Py_ssize_t refcnt, size;
  void* lookup;
  Py_ssize_t usable, nentries;
  char idx[1];
};
inline const DkEntry* dk_entries(PyObject* o, Py_ssize_t& n) {
  n = 0;
  if (Py_TYPE(o) != &PyDict_Type) return nullptr;
  const PyDictObject* d = (const PyDictObject*)o;
  if (d->ma_values) return nullptr;  // split table
  const DkHead* k = (const DkHead*)d->ma_keys;
  const Py_ssize_t sz = k->size;
  const int ix = sz <= 0xff ? 1 : sz <= 0xffff ? 2 : sz <= 0xffffffffLL ? 4 : 8;
  n = k->nentries;
  return (const DkEntry*)(k->idx + sz * ix);
}
#define EDV_HAVE_DK 1
#endif
bool g_scan_direct = true;  // EDV_SCAN_DIRECT=0: PyDict_Next instead (A/B); set per scan call
inline bool g_scan_direct_env() {
  const char* e = getenv("EDV_SCAN_DIRECT");
  return !(e && e[0] == '0');
}

bool w_str_eq(PyObject* a, PyObject* b) {  // canonical kinds: equal strings have equal kinds
  const Py_ssize_t n = PyUnicode_GET_LENGTH(a);
  return PyUnicode_KIND(a) == PyUnicode_KIND(b) && n == PyUnicode_GET_LENGTH(b) &&
         memcmp(PyUnicode_DATA(a), PyUnicode_DATA(b), (size_t)n * PyUnicode_KIND(a)) == 0;
}

bool w_ignored(PyObject* k, PyObject* ignore) {
  if (!ignore) return false;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(ignore);
  PyObject** items = PySequence_Fast_ITEMS(ignore);
  for (Py_ssize_t i = 0; i < n; ++i)
    if (PyUnicode_CheckExact(items[i]) && w_str_eq(k, items[i])) return true;
  return false;
}

bool w_less(PyObject* a, PyObject* b) {  // both one-byte kind (checked by the caller)
  const Py_ssize_t na = PyUnicode_GET_LENGTH(a), nb = PyUnicode_GET_LENGTH(b);
  const unsigned char *pa = PyUnicode_1BYTE_DATA(a), *pb = PyUnicode_1BYTE_DATA(b);
  if (na && nb && pa[0] != pb[0]) return pa[0] < pb[0];  // most keys differ in their first byte
  const int c = memcmp(pa, pb, (size_t)(na < nb ? na : nb));
  return c < 0 || (c == 0 && na < nb);
}

WRes w_append_str(PyObject* s, OutBuf& out) {
  if (!PyUnicode_IS_ASCII(s)) return kDefer;  // UTF-8 encoding may allocate
  out.append((const char*)PyUnicode_1BYTE_DATA(s), (size_t)PyUnicode_GET_LENGTH(s));
  return kOk;
}

// top != nullptr (a request's top level): also hands back the values of the keys top[0]
// (signature) and top[1] (identifier) in found[0..1], from the same pass over the dict; both
// null when the dict has a non-str key (the item then takes the Python path).
WRes wser_dict(PyObject* d, int level, PyObject* ignore, OutBuf& out, PyObject* const* top = nullptr,
               PyObject** found = nullptr) {
  constexpr Py_ssize_t kSmall = 24;
  struct KV {
    PyObject *k, *v;
  };
  KV small[kSmall];
  std::vector<KV> big;
  const Py_ssize_t nd = PyDict_GET_SIZE(d);
  KV* kv = small;
  if (nd > kSmall) {
    big.resize((size_t)nd);
    kv = big.data();
  }
  Py_ssize_t nk = 0;
  bool one_byte = true;
  const auto take = [&](PyObject* k, PyObject* v) -> bool {  // false: a non-str key
    if (!PyUnicode_CheckExact(k)) {
      if (top) found[0] = found[1] = nullptr;
      return false;  // as ser_dict
    }
    if (top) {
      if (k == top[0] || w_str_eq(k, top[0]))
        found[0] = v;
      else if (k == top[1] || w_str_eq(k, top[1]))
        found[1] = v;
    }
    if (level == 0 && w_ignored(k, ignore)) return true;
    one_byte = one_byte && PyUnicode_KIND(k) == PyUnicode_1BYTE_KIND;
    kv[nk++] = KV{k, v};
    return true;
  };
#ifdef EDV_HAVE_DK
  Py_ssize_t ne = 0;
  const DkEntry* ent = g_scan_direct ? dk_entries(d, ne) : nullptr;
  if (ent) {
    for (Py_ssize_t e = 0; e < ne; ++e)  // insertion order, deleted entries (value NULL) skipped
      if (ent[e].v && !take(ent[e].k, ent[e].v)) return kFail;
  } else
#endif
  {
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(d, &pos, &k, &v))
      if (!take(k, v)) return kFail;
  }
  if (!one_byte) return kDefer;  // PyUnicode_Compare order for wider kinds: ser_dict
  if (nk <= kSmall) {  // insertion sort: a request's dicts have a handful of keys
    for (Py_ssize_t i = 1; i < nk; ++i) {
      const KV x = kv[i];
      Py_ssize_t j = i;
      while (j > 0 && w_less(x.k, kv[j - 1].k)) {
        kv[j] = kv[j - 1];
        --j;
      }
      kv[j] = x;
    }
  } else {
    std::sort(kv, kv + nk, [](const KV& a, const KV& b) { return w_less(a.k, b.k); });
  }
  for (Py_ssize_t i = 0; i < nk; ++i) {
    if (i) out.push_back('|');
    WRes r = w_append_str(kv[i].k, out);
    if (r != kOk) return r;
    out.push_back(':');
    r = wser_obj(kv[i].v, level + 1, nullptr, out);
    if (r != kOk) return r;
  }
  return kOk;
}

// An exact int's value when it has at most two 30-bit digits (CPython's long layout up to
// 3.11), without the out-of-line PyLong_AsLongLongAndOverflow call; false: use the API.
inline bool w_small_long(PyObject* o, long long& x) {
#if PY_VERSION_HEX < 0x030C0000 && PYLONG_BITS_IN_DIGIT == 30
  const Py_ssize_t sz = Py_SIZE(o);
  const digit* dg = ((PyLongObject*)o)->ob_digit;
  if (sz == 0) {
    x = 0;
    return true;
  }
  const Py_ssize_t a = sz < 0 ? -sz : sz;
  if (a > 2) return false;
  long long v = (long long)dg[0];
  if (a == 2) v |= (long long)dg[1] << 30;
  x = sz < 0 ? -v : v;
  return true;
#else
  (void)o;
  (void)x;
  return false;
#endif
}

WRes wser_obj(PyObject* o, int level, PyObject* ignore, OutBuf& out) {
  if (level > kMaxDepth) return kFail;
  if (PyUnicode_CheckExact(o)) return w_append_str(o, out);
  if (PyDict_CheckExact(o)) return wser_dict(o, level, ignore, out);
  if (PyList_CheckExact(o)) {
    const Py_ssize_t n = PyList_GET_SIZE(o);
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) out.push_back(',');
      const WRes r = wser_obj(PyList_GET_ITEM(o, i), level + 1, nullptr, out);
      if (r != kOk) return r;
    }
    return kOk;
  }
  if (o == Py_None) return kOk;
  if (PyBool_Check(o)) {
    out.append(o == Py_True ? "True" : "False");
    return kOk;
  }
  if (PyLong_CheckExact(o)) {
    long long x;
    if (!w_small_long(o, x)) {
      int overflow = 0;
      x = PyLong_AsLongLongAndOverflow(o, &overflow);  // an exact int never errors
      if (overflow) return kDefer;
    }
    char b[24];
    const auto r = std::to_chars(b, b + sizeof b, x);
    out.append_short(b, (size_t)(r.ptr - b));
    return kOk;
  }
  if (PyFloat_CheckExact(o)) return kDefer;  // Python's repr: str() under the GIL
  return kFail;
}

// ------------------------------------------------ shape-cached serialization
// Requests from one client library have the same keys in the same insertion order, batch after
// batch (a NYM: identifier, reqId, operation {type, dest, verkey, alias}, protocolVersion,
// signature).  Each scan worker remembers, per nesting class and entry count, the last dict
// "shape" it serialized generically: its key texts in insertion order, the order the serializer
// emits them in (sorted, level-0 ignored keys dropped), the "|key:" prefixes, and where the
// signature / identifier entries sit.  A dict whose keys match a remembered shape text for text
// (exact compact-ASCII str keys, no deleted entries) is emitted from it: no per-key ignore or
// top-key comparisons, no sort, one prefix copy per key.  Anything else takes wser_dict (which
// then remembers the new shape).  The bytes are wser_dict's in every case (tests/
// test_hostpack.py: shapes on / off / the Python restatement over a pool of near-miss shapes).
#ifdef EDV_HAVE_DK
constexpr int kShapeKeys = 12;     // dicts with more entries: wser_dict
constexpr size_t kShapeKeyLen = 40;  // longer keys: wser_dict
struct ShapeKey {
  uint32_t len = 0;
  uint64_t a = 0, b = 0;  // the text's first and last 8 (or 4) bytes (keys of up to 16 bytes)
  const char* txt = nullptr;
};
inline uint64_t ld8(const char* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
inline uint32_t ld4(const char* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline void key_words(const char* p, size_t n, uint64_t& a, uint64_t& b) {
  if (n >= 8) {
    a = ld8(p), b = ld8(p + n - 8);
  } else if (n >= 4) {
    a = ld4(p), b = ld4(p + n - 4);
  } else {
    a = n ? (uint64_t)(unsigned char)p[0] | (uint64_t)(unsigned char)p[n / 2] << 8 |
                (uint64_t)(unsigned char)p[n - 1] << 16
          : 0;
    b = 0;
  }
}
// k is an exact, compact ASCII str whose text is sk's
inline bool key_is(const ShapeKey& sk, PyObject* k) {
  if (Py_TYPE(k) != &PyUnicode_Type) return false;
  const PyASCIIObject* o = (const PyASCIIObject*)k;
  if (!o->state.compact || !o->state.ascii || (uint32_t)o->length != sk.len) return false;
  const char* p = (const char*)(o + 1);
  if (sk.len > 16) return memcmp(p, sk.txt, sk.len) == 0;
  uint64_t a, b;
  key_words(p, sk.len, a, b);
  return a == sk.a && b == sk.b;
}
struct Shape {
  int ne = -1;  // entries; -1: empty
  ShapeKey key[kShapeKeys];
  uint8_t emit[kShapeKeys];  // entry index of each emitted key, in emit order
  uint8_t pre_len[kShapeKeys];
  uint16_t pre_at[kShapeKeys];
  int nemit = 0;
  int8_t sig_at = -1, idr_at = -1;  // level 0: the entries holding the signature / identifier
  char text[kShapeKeys * (kShapeKeyLen + 2)];
  char pre[kShapeKeys * (kShapeKeyLen + 2)];
};
struct ShapeCache {
  Shape s[2][8];  // [level 0 / deeper][entries % 8]
  Shape& at(int level, Py_ssize_t ne) { return s[level ? 1 : 0][ne & 7]; }
};

WRes shaped_dict(PyObject* d, int level, PyObject* ignore, OutBuf& out, PyObject* const* top, PyObject** found,
                 ShapeCache& sc);

inline WRes shaped_val(PyObject* v, int level, OutBuf& out, ShapeCache& sc) {
  PyTypeObject* t = Py_TYPE(v);
  if (t == &PyUnicode_Type) {
    const PyASCIIObject* o = (const PyASCIIObject*)v;
    if (o->state.compact && o->state.ascii) {
      out.append((const char*)(o + 1), (size_t)o->length);
      return kOk;
    }
    return w_append_str(v, out);
  }
  if (t == &PyDict_Type) return shaped_dict(v, level, nullptr, out, nullptr, nullptr, sc);
  return wser_obj(v, level, nullptr, out);
}

// remember d's shape (after wser_dict serialized it with kOk): every key an exact compact ASCII
// str of at most kShapeKeyLen bytes, at most kShapeKeys entries, none deleted
void shape_learn(Shape& sh, const DkEntry* ent, Py_ssize_t ne, int level, PyObject* ignore, PyObject* const* top) {
  sh.ne = -1;
  if (ne > kShapeKeys) return;
  size_t tat = 0;
  int keep[kShapeKeys];
  int nk = 0;
  sh.sig_at = sh.idr_at = -1;
  for (Py_ssize_t j = 0; j < ne; ++j) {
    PyObject* k = ent[j].k;
    if (!ent[j].v || Py_TYPE(k) != &PyUnicode_Type) return;
    const PyASCIIObject* o = (const PyASCIIObject*)k;
    if (!o->state.compact || !o->state.ascii || (size_t)o->length > kShapeKeyLen) return;
    ShapeKey& sk = sh.key[j];
    sk.len = (uint32_t)o->length;
    memcpy(sh.text + tat, (const char*)(o + 1), sk.len);
    sk.txt = sh.text + tat;
    tat += sk.len;
    key_words(sk.txt, sk.len, sk.a, sk.b);
    if (top) {
      if (k == top[0] || w_str_eq(k, top[0]))
        sh.sig_at = (int8_t)j;
      else if (k == top[1] || w_str_eq(k, top[1]))
        sh.idr_at = (int8_t)j;
    }
    if (level == 0 && w_ignored(k, ignore)) continue;
    keep[nk++] = (int)j;
  }
  for (int i = 1; i < nk; ++i) {  // wser_dict's order
    const int x = keep[i];
    int j = i;
    while (j > 0 && w_less(ent[x].k, ent[keep[j - 1]].k)) {
      keep[j] = keep[j - 1];
      --j;
    }
    keep[j] = x;
  }
  size_t pat = 0;
  for (int i = 0; i < nk; ++i) {
    const ShapeKey& sk = sh.key[keep[i]];
    sh.emit[i] = (uint8_t)keep[i];
    sh.pre_at[i] = (uint16_t)pat;
    if (i) sh.pre[pat++] = '|';
    memcpy(sh.pre + pat, sk.txt, sk.len);
    pat += sk.len;
    sh.pre[pat++] = ':';
    sh.pre_len[i] = (uint8_t)(pat - sh.pre_at[i]);
  }
  sh.nemit = nk;
  sh.ne = (int)ne;
}

WRes shaped_dict(PyObject* d, int level, PyObject* ignore, OutBuf& out, PyObject* const* top, PyObject** found,
                 ShapeCache& sc) {
  if (level > kMaxDepth) return kFail;
  Py_ssize_t ne = 0;
  const DkEntry* ent = dk_entries(d, ne);
  if (!ent || ne != ((PyDictObject*)d)->ma_used) return wser_dict(d, level, ignore, out, top, found);
  Shape& sh = sc.at(level, ne);
  bool hit = sh.ne == ne;
  for (Py_ssize_t j = 0; hit && j < ne; ++j) hit = key_is(sh.key[j], ent[j].k);
  if (!hit) {
    const WRes r = wser_dict(d, level, ignore, out, top, found);
    if (r == kOk) shape_learn(sh, ent, ne, level, ignore, top);
    return r;
  }
  if (top) {
    found[0] = sh.sig_at >= 0 ? ent[sh.sig_at].v : nullptr;
    found[1] = sh.idr_at >= 0 ? ent[sh.idr_at].v : nullptr;
  }
  for (int i = 0; i < sh.nemit; ++i) {
    out.append(sh.pre + sh.pre_at[i], sh.pre_len[i]);
    const WRes r = shaped_val(ent[sh.emit[i]].v, level + 1, out, sc);
    if (r != kOk) return r;
  }
  return kOk;
}
#endif

// ------------------------------------------------------------------- base58

const char kAlphabet[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

struct B58Index {
  int8_t v[256];
  B58Index() {
    memset(v, -1, sizeof v);
    for (int i = 0; i < 58; ++i) v[(unsigned char)kAlphabet[i]] = (int8_t)i;
  }
};
const B58Index kIndex;

// false on a character outside the alphabet.  Base conversion on 64-bit
// limbs, ten base-58 digits (58^10 < 2^59) per multiply-add pass with 128-bit
// products (an 88-character signature: 9 passes over at most 4 limbs).
bool b58decode_raw(const unsigned char* s, size_t n, std::vector<uint8_t>& out) {
  size_t nz = 0;
  while (nz < n && s[nz] == '1') ++nz;
  uint64_t stack_limbs[16];
  std::vector<uint64_t> heap;
  uint64_t* limb = stack_limbs;
  const size_t cap = (n - nz) / 10 + 2;
  if (cap > 16) {
    heap.resize(cap);
    limb = heap.data();
  }
  size_t nl = 0, i = nz;
  while (i < n) {
    uint64_t mul = 1, chunk = 0;
    for (int k = 0; k < 10 && i < n; ++k, ++i) {
      const int d = kIndex.v[s[i]];
      if (d < 0) return false;
      chunk = chunk * 58u + (uint64_t)d;
      mul *= 58u;
    }
    unsigned __int128 carry = chunk;
    for (size_t j = 0; j < nl; ++j) {
      const unsigned __int128 t = (unsigned __int128)limb[j] * mul + carry;
      limb[j] = (uint64_t)t;
      carry = t >> 64;
    }
    if (carry) limb[nl++] = (uint64_t)carry;
  }
  // big-endian bytes of the number without its leading zero bytes, after nz zero bytes
  size_t top = nl ? 8 - (size_t)(__builtin_clzll(limb[nl - 1]) >> 3) : 0;  // bytes of the top limb
  const size_t len = nl ? top + (nl - 1) * 8 : 0;
  out.resize(nz + len);
  uint8_t* o = out.data();
  memset(o, 0, nz);
  o += nz;
  for (size_t j = nl; j-- > 0;) {
    const size_t nb = j == nl - 1 ? top : 8;
    for (size_t b = 0; b < nb; ++b) *o++ = (uint8_t)(limb[j] >> (8 * (nb - 1 - b)));
  }
  return true;
}

// base58 0.2.4 b58encode: leading zero bytes -> '1's, the rest as a
// big-endian base-58 number (repeated division of the byte string).
std::string b58encode_raw(const uint8_t* v, size_t n) {
  static const char kAlpha[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
  size_t nz = 0;
  while (nz < n && v[nz] == 0) ++nz;
  std::vector<uint8_t> num(v + nz, v + n);
  std::string digits;
  size_t start = 0;
  while (start < num.size()) {
    uint32_t rem = 0;
    for (size_t i = start; i < num.size(); ++i) {
      const uint32_t cur = rem * 256 + num[i];
      num[i] = (uint8_t)(cur / 58);
      rem = cur % 58;
    }
    digits.push_back(kAlpha[rem]);
    while (start < num.size() && num[start] == 0) ++start;
  }
  return std::string(nz, '1') + std::string(digits.rbegin(), digits.rend());
}

// Signature slots (edverify.h EDV_SIG_SLOT96): a signature whose base58 text
// decodes to exactly 64 bytes travels as its text and is decoded on the GPU
// (edv_b58_sig_kernel); the host only needs to know that the decoded length
// is 64, because crypto_sign_open's split of sig || ser at byte 64
// (nacl_wrappers.py:108) depends on it.  The text after its nz leading '1's
// (zero bytes) is a number whose byte length must be L = 64 - nz, i.e.
// 256^(L-1) <= value < 256^L; base58 digits are in ASCII order, so for texts
// of equal length the numeric comparison is memcmp against the encodings of
// those powers.
struct B58Len64 {
  std::string lo[65], hi[65];  // L = 1..64: b58(256^(L-1)), b58(256^L)
  B58Len64() {
    std::vector<uint8_t> v(66, 0);
    v[0] = 1;
    for (size_t L = 1; L <= 64; ++L) {
      lo[L] = b58encode_raw(v.data(), L);
      hi[L] = b58encode_raw(v.data(), L + 1);
    }
  }
};
const B58Len64& b58_len64_table() {
  static const B58Len64 t;
  return t;
}

// Every character in the base58 alphabet (1-9 A-H J-N P-Z a-k m-z): 16 at a time as six
// unsigned range tests (SSE2, part of x86-64), the tail by the table.
bool b58_chars_ok(const unsigned char* s, size_t n) {
  size_t i = 0;
  for (; i + 16 <= n; i += 16) {
    const __m128i c = _mm_loadu_si128((const __m128i*)(s + i));
    auto in = [&c](char lo, char hi) {
      const __m128i x = _mm_sub_epi8(c, _mm_set1_epi8(lo));
      return _mm_cmpeq_epi8(_mm_min_epu8(x, _mm_set1_epi8((char)(hi - lo))), x);  // x <= hi - lo (unsigned)
    };
    const __m128i ok = _mm_or_si128(_mm_or_si128(_mm_or_si128(in('1', '9'), in('A', 'H')), in('J', 'N')),
                                    _mm_or_si128(_mm_or_si128(in('P', 'Z'), in('a', 'k')), in('m', 'z')));
    if (_mm_movemask_epi8(ok) != 0xFFFF) return false;
  }
  for (; i < n; ++i)
    if (kIndex.v[s[i]] < 0) return false;
  return true;
}

// 1: b58decode(s) is valid and exactly 64 bytes; 0: valid, another length;
// -1: a character outside the alphabet (b58decode raises).
int b58_len64(const unsigned char* s, size_t n) {
  if (!b58_chars_ok(s, n)) return -1;
  size_t nz = 0;
  while (nz < n && s[nz] == '1') ++nz;
  if (nz > 64) return 0;
  const size_t L = 64 - nz, d = n - nz;
  if (L == 0) return d == 0 ? 1 : 0;
  if (d == 0) return 0;  // the value is 0: nz < 64 zero bytes
  const B58Len64& t = b58_len64_table();
  const std::string &lo = t.lo[L], &hi = t.hi[L];
  const unsigned char* r = s + nz;
  const bool ge = d > lo.size() || (d == lo.size() && memcmp(r, lo.data(), d) >= 0);
  const bool lt = d < hi.size() || (d == hi.size() && memcmp(r, hi.data(), d) < 0);
  return ge && lt ? 1 : 0;
}

PyObject* py_b58_len64(PyObject*, PyObject* v) {
  if (!PyUnicode_CheckExact(v) || !PyUnicode_IS_ASCII(v)) {
    PyErr_SetString(PyExc_TypeError, "ASCII str expected");
    return nullptr;
  }
  return PyLong_FromLong(b58_len64(PyUnicode_1BYTE_DATA(v), (size_t)PyUnicode_GET_LENGTH(v)));
}

// b58encode_rows(buf, width) -> [b58encode(buf[i*width:(i+1)*width]) ...]
PyObject* py_b58encode_rows(PyObject*, PyObject* args) {
  Py_buffer b;
  Py_ssize_t width;
  if (!PyArg_ParseTuple(args, "y*n", &b, &width)) return nullptr;
  if (width <= 0 || b.len % width) {
    PyBuffer_Release(&b);
    PyErr_SetString(PyExc_ValueError, "buffer length is not a multiple of width");
    return nullptr;
  }
  const Py_ssize_t rows = b.len / width;
  PyObject* out = PyList_New(rows);
  if (!out) {
    PyBuffer_Release(&b);
    return nullptr;
  }
  for (Py_ssize_t i = 0; i < rows; ++i) {
    const std::string e = b58encode_raw((const uint8_t*)b.buf + i * width, (size_t)width);
    PyObject* str = PyUnicode_FromStringAndSize(e.data(), (Py_ssize_t)e.size());
    if (!str) {
      Py_DECREF(out);
      PyBuffer_Release(&b);
      return nullptr;
    }
    PyList_SET_ITEM(out, i, str);
  }
  PyBuffer_Release(&b);
  return out;
}

PyObject* py_b58decode(PyObject*, PyObject* v) {
  const unsigned char* s = nullptr;
  Py_ssize_t n = 0;
  if (PyUnicode_CheckExact(v)) {
    if (!PyUnicode_IS_ASCII(v)) Py_RETURN_NONE;  // the reference raises ValueError
    s = (const unsigned char*)PyUnicode_AsUTF8AndSize(v, &n);
    if (!s) return nullptr;
  } else if (PyBytes_CheckExact(v)) {
    s = (const unsigned char*)PyBytes_AS_STRING(v);
    n = PyBytes_GET_SIZE(v);
    for (Py_ssize_t i = 0; i < n; ++i)
      if (s[i] >= 0x80) Py_RETURN_NONE;  // .decode('ascii') raises in the reference
  } else {
    Py_RETURN_NONE;
  }
  std::vector<uint8_t> out;
  if (!b58decode_raw(s, (size_t)n, out)) Py_RETURN_NONE;
  return PyBytes_FromStringAndSize((const char*)out.data(), (Py_ssize_t)out.size());
}

// ------------------------------------------------------------------ packing

bool bytes_of(PyObject* o, const char** p, Py_ssize_t* n) {
  if (!PyBytes_Check(o)) {
    PyErr_SetString(PyExc_TypeError, "bytes expected");
    return false;
  }
  *p = PyBytes_AS_STRING(o);
  *n = PyBytes_GET_SIZE(o);
  return true;
}

PyObject* py_pack_split64(PyObject*, PyObject* args) {
  PyObject *sigs, *sers;
  if (!PyArg_ParseTuple(args, "OO", &sigs, &sers)) return nullptr;
  PyObject* fs = PySequence_Fast(sigs, "sigs must be a sequence");
  if (!fs) return nullptr;
  PyObject* fm = PySequence_Fast(sers, "sers must be a sequence");
  if (!fm) {
    Py_DECREF(fs);
    return nullptr;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fs);
  PyObject* ret = nullptr;
  if (PySequence_Fast_GET_SIZE(fm) != n) {
    PyErr_SetString(PyExc_ValueError, "length mismatch");
  } else {
    std::string sig64((size_t)n * 64, '\0'), msgs, shortv((size_t)n, '\0');
    std::vector<uint64_t> off((size_t)n + 1, 0);
    bool ok = true;
    for (Py_ssize_t i = 0; i < n && ok; ++i) {
      const char *s, *m;
      Py_ssize_t ns, nm;
      ok = bytes_of(PySequence_Fast_GET_ITEM(fs, i), &s, &ns) && bytes_of(PySequence_Fast_GET_ITEM(fm, i), &m, &nm);
      if (!ok) break;
      if (ns + nm < 64) {
        shortv[(size_t)i] = 1;  // crypto_sign_open: smlen < 64 rejects
      } else if (ns >= 64) {
        memcpy(&sig64[(size_t)i * 64], s, 64);
        msgs.append(s + 64, (size_t)(ns - 64));  // sm[64:] = sig[64:] || ser
        msgs.append(m, (size_t)nm);
      } else {
        memcpy(&sig64[(size_t)i * 64], s, (size_t)ns);
        memcpy(&sig64[(size_t)i * 64 + ns], m, (size_t)(64 - ns));
        msgs.append(m + (64 - ns), (size_t)(nm - (64 - ns)));
      }
      off[(size_t)i + 1] = msgs.size();
    }
    if (ok)
      ret = Py_BuildValue("(y#y#y#y#)", sig64.data(), (Py_ssize_t)sig64.size(), msgs.data(), (Py_ssize_t)msgs.size(),
                          (const char*)off.data(), (Py_ssize_t)(off.size() * 8), shortv.data(),
                          (Py_ssize_t)shortv.size());
  }
  Py_DECREF(fs);
  Py_DECREF(fm);
  return ret;
}

PyObject* py_pack_sm(PyObject*, PyObject* args) {
  PyObject *sigs, *sers, *keys;
  if (!PyArg_ParseTuple(args, "OOO", &sigs, &sers, &keys)) return nullptr;
  PyObject* fs = PySequence_Fast(sigs, "sigs must be a sequence");
  PyObject* fm = fs ? PySequence_Fast(sers, "sers must be a sequence") : nullptr;
  PyObject* fk = fm ? PySequence_Fast(keys, "keys must be a sequence") : nullptr;
  PyObject* ret = nullptr;
  if (fk) {
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fs);
    if (PySequence_Fast_GET_SIZE(fm) != n || PySequence_Fast_GET_SIZE(fk) != n) {
      PyErr_SetString(PyExc_ValueError, "length mismatch");
    } else {
      std::string sm, pk((size_t)n * 32, '\0');
      std::vector<uint64_t> off((size_t)n + 1, 0);
      bool ok = true;
      for (Py_ssize_t i = 0; i < n && ok; ++i) {
        const char *s, *m, *k;
        Py_ssize_t ns, nm, nk;
        ok = bytes_of(PySequence_Fast_GET_ITEM(fs, i), &s, &ns) && bytes_of(PySequence_Fast_GET_ITEM(fm, i), &m, &nm) &&
             bytes_of(PySequence_Fast_GET_ITEM(fk, i), &k, &nk);
        if (!ok) break;
        if (nk != 32) {
          PyErr_SetString(PyExc_ValueError, "keys must be 32 bytes");
          ok = false;
          break;
        }
        sm.append(s, (size_t)ns);
        sm.append(m, (size_t)nm);
        off[(size_t)i + 1] = sm.size();
        memcpy(&pk[(size_t)i * 32], k, 32);
      }
      if (ok)
        ret = Py_BuildValue("(y#y#y#)", sm.data(), (Py_ssize_t)sm.size(), (const char*)off.data(),
                            (Py_ssize_t)(off.size() * 8), pk.data(), (Py_ssize_t)pk.size());
    }
  }
  Py_XDECREF(fs);
  Py_XDECREF(fm);
  Py_XDECREF(fk);
  return ret;
}

// scan_batch(msgs, ignore[, threads]) -> (fast, idrs, sig64, msgbuf, off, short)
// scan_batch_u(msgs, ignore[, threads]) -> (fast, uidx, uniq, sig64, msgbuf, off, short)
// The host half of NaclAuthNr.authenticate for a batch of request dicts
// (client_authn.py:72-92) where every step succeeds without a decision the
// Python code must make: msg[signature] is a non-empty str, msg[identifier] a
// non-empty str, b58decode(signature) succeeds and serialize_for_signing takes
// its native path.  For those items (fast[i] = 1) the signed stream
// sm = b58decode(sig) || ser is split at byte 64 like crypto_sign_open
// (nacl_wrappers.py:108): sig64 (n * 64), messages (msgbuf + off[n + 1],
// uint64 LE), short[i] = len(sm) < 64.  idrs[i] is the identifier (fast items)
// or None; the _u form gives instead uidx[i] (uint32 LE, 0xffffffff for
// non-fast items) into uniq, the batch's distinct identifiers, so the caller
// resolves each verkey once without a per-item loop.
// Every other item (fast[i] = 0, zero-length slots) takes the Python
// _prepare, which raises the reference's exception.
//
// Phases: (1) `threads` workers (0 = auto) split the items into ranges and do
// the checks, the base58 decode, the serialization (wser_obj) and the
// identifier's slot into tables of their own, reading objects only as
// wser_obj does; (2) the identifier tables merged; (3) under the GIL, the
// items the workers could not finish (ser_obj); (4) offsets by prefix sum;
// (5) the workers write sig64 and the message buffer straight into the result
// bytes objects.
constexpr int kSigSlot = 96;  // edverify.h EDV_SIG_SLOT96

// The batch's distinct identifiers: an open-addressing table over the
// identifier text (a 64-bit multiply-xor hash of 8-byte words, linear
// probing, grown at half load).  Every request carries its identifier as its
// own str object (json-decoded from the wire), so the lookup is by content.
// A node-based std::unordered_map<std::string_view> here allocated a node per
// emplace and cost ~30 % of a worker's time per request.
struct IdrTable {
  // an identifier of up to kInl bytes is compared against a copy in its entry (one cache line),
  // not against the first object's data, which a churning batch's ~30k identifiers leave cold
  static constexpr size_t kInl = 32;
  struct alignas(64) E {
    uint64_t h;
    const char* p;  // the identifier's bytes (the str object's data; owned by the batch's dicts)
    size_t n;
    uint32_t id;
    char inl[kInl];  // (n <= kInl) a copy of them
  };
  std::vector<E> e;
  size_t mask = 0, used = 0;
  static uint64_t hash(const char* p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      memcpy(&w, p + i, 8);
      h = (h ^ w) * 0xff51afd7ed558ccdull;
      h ^= h >> 32;
    }
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = (h ^ w) * 0xc4ceb9fe1a85ec53ull;
    return h ^ (h >> 29);
  }
  void reset(size_t expect) {
    size_t cap = 64;
    while (cap < 2 * expect) cap <<= 1;
    e.assign(cap, E{});
    mask = cap - 1;
    used = 0;
  }
  // the id of text (p, n), or `next` (fresh = true) when it is new
  uint32_t find_or_add(const char* p, size_t n, uint32_t next, bool& fresh) {
    return find_or_add_h(hash(p, n), p, n, next, fresh);
  }
  uint32_t find_or_add_h(uint64_t h, const char* p, size_t n, uint32_t next, bool& fresh) {  // h = hash(p, n)
    if (2 * (used + 1) > e.size()) grow();
    for (size_t s = h & mask;; s = (s + 1) & mask) {
      E& x = e[s];
      if (!x.p) {
        x.h = h, x.p = p, x.n = n, x.id = next;
        if (n <= kInl) memcpy(x.inl, p, n);
        ++used;
        fresh = true;
        return next;
      }
      if (x.h == h && x.n == n && (x.p == p || memcmp(n <= kInl ? x.inl : x.p, p, n) == 0)) {
        fresh = false;
        return x.id;
      }
    }
  }
  void grow() {
    std::vector<E> old;
    old.swap(e);
    e.assign(old.empty() ? 64 : old.size() * 2, E{});
    mask = e.size() - 1;
    for (const E& x : old)
      if (x.p)
        for (size_t s = x.h & mask;; s = (s + 1) & mask)
          if (!e[s].p) {
            e[s] = x;
            break;
          }
  }
};

// Identifier text -> key-store id, from the batches before (the authenticator's speculation
// for a staged batch: the scan writes each request's key id while it scans, so the batch's
// kernels can run under the scan; the authenticator checks every id against getVerkey and
// the key store afterwards).  Owns copies of the texts.
struct KidMap {
  struct E {
    uint64_t h = 0;
    uint32_t off = 0, len = 0, kid = 0;
    bool used = false;
  };
  std::vector<E> e;
  std::string text;
  size_t used = 0;
  KidMap() { e.resize(1024); }
  uint32_t get(const char* p, size_t n) const {
    const size_t mask = e.size() - 1;
    const uint64_t h = IdrTable::hash(p, n);
    for (size_t s = h & mask;; s = (s + 1) & mask) {
      const E& x = e[s];
      if (!x.used) return 0xffffffffu;
      if (x.h == h && x.len == n && memcmp(text.data() + x.off, p, n) == 0) return x.kid;
    }
  }
  void put(const char* p, size_t n, uint32_t kid) {
    if (2 * (used + 1) > e.size()) {
      std::vector<E> old;
      old.swap(e);
      e.resize(old.size() * 2);
      for (const E& x : old)
        if (x.used)
          for (size_t s = x.h & (e.size() - 1);; s = (s + 1) & (e.size() - 1))
            if (!e[s].used) {
              e[s] = x;
              break;
            }
    }
    const size_t mask = e.size() - 1;
    const uint64_t h = IdrTable::hash(p, n);
    for (size_t s = h & mask;; s = (s + 1) & mask) {
      E& x = e[s];
      if (!x.used) {
        x.h = h, x.off = (uint32_t)text.size(), x.len = (uint32_t)n, x.kid = kid, x.used = true;
        text.append(p, n);
        ++used;
        return;
      }
      if (x.h == h && x.len == n && memcmp(text.data() + x.off, p, n) == 0) {
        x.kid = kid;  // (an id that is no longer right: ~0u, so the scan writes "unknown")
        return;
      }
    }
  }
};
void kid_map_free(PyObject* cap) { delete (KidMap*)PyCapsule_GetPointer(cap, "edv.kidmap"); }

// kid_map(old, identifiers, ids) -> map: old (a kid_map or None) with identifiers[j] -> ids[j]
// (uint32 bytes; 0xffffffff = no id) put; a new map when old is None.  ASCII identifiers only
// (others are skipped: the scan defers their requests anyway).
PyObject* py_kid_map(PyObject*, PyObject* args) {
  PyObject *old, *idrs;
  Py_buffer bk;
  if (!PyArg_ParseTuple(args, "OOy*", &old, &idrs, &bk)) return nullptr;
  struct Rel {
    Py_buffer* b;
    ~Rel() { PyBuffer_Release(b); }
  } rel{&bk};
  if (!PyList_CheckExact(idrs) || bk.len != PyList_GET_SIZE(idrs) * 4) {
    PyErr_SetString(PyExc_ValueError, "kid_map: a list of identifiers and as many uint32 ids");
    return nullptr;
  }
  KidMap* m = nullptr;
  PyObject* ret = nullptr;
  if (old == Py_None) {
    m = new KidMap;
    ret = PyCapsule_New(m, "edv.kidmap", kid_map_free);
    if (!ret) {
      delete m;
      return nullptr;
    }
  } else {
    m = (KidMap*)PyCapsule_GetPointer(old, "edv.kidmap");
    if (!m) return nullptr;
    Py_INCREF(old);
    ret = old;
  }
  const uint32_t* k = (const uint32_t*)bk.buf;
  for (Py_ssize_t j = 0; j < PyList_GET_SIZE(idrs); ++j) {
    PyObject* o = PyList_GET_ITEM(idrs, j);
    if (PyUnicode_CheckExact(o) && PyUnicode_IS_ASCII(o))
      m->put((const char*)PyUnicode_1BYTE_DATA(o), (size_t)PyUnicode_GET_LENGTH(o), k[j]);
  }
  return ret;
}
// verify_one(fn, ctx, sig64, key_id, msg) -> bool: edverify.h edv_verify_one through its address
// (EdVerifyEngine.verify_one_keyed's call without the ctypes argument conversions: the per-message
// authenticate() that missed the verify-ahead cache), the GIL released while the GPU answers.
// Raises RuntimeError(code) when the library returns an error (the caller reads edv_last_error).
using VerifyOneFn = int (*)(void*, const uint8_t*, uint32_t, const uint8_t*, uint64_t, uint8_t*);
PyObject* py_verify_one(PyObject*, PyObject* args) {
  unsigned long long fn, ctx;
  Py_buffer sig, msg;
  unsigned int kid;
  if (!PyArg_ParseTuple(args, "KKy*Iy*", &fn, &ctx, &sig, &kid, &msg)) return nullptr;
  int r = -1;
  uint8_t ok = 0;
  if (sig.len != 64 || !fn || !ctx) {
    PyBuffer_Release(&sig);
    PyBuffer_Release(&msg);
    PyErr_SetString(PyExc_ValueError, "verify_one: a 64-byte signature and the library's addresses");
    return nullptr;
  }
  Py_BEGIN_ALLOW_THREADS
  r = ((VerifyOneFn)(uintptr_t)fn)((void*)(uintptr_t)ctx, (const uint8_t*)sig.buf, (uint32_t)kid,
                                   msg.len ? (const uint8_t*)msg.buf : nullptr, (uint64_t)msg.len, &ok);
  Py_END_ALLOW_THREADS
  PyBuffer_Release(&sig);
  PyBuffer_Release(&msg);
  if (r != 0) {
    PyErr_Format(PyExc_RuntimeError, "edv_verify_one %d", r);
    return nullptr;
  }
  return PyBool_FromLong(ok & 1);
}

PyObject* py_kid_map_size(PyObject*, PyObject* cap) {
  KidMap* m = (KidMap*)PyCapsule_GetPointer(cap, "edv.kidmap");
  return m ? PyLong_FromSize_t(m->used) : nullptr;
}

// Writes into the engine's pinned memory that only the DMA reads back: non-temporal stores
// (no read-for-ownership of the destination lines, nothing evicted from the worker's cache).
// The caller fences (_mm_sfence) before publishing what it wrote to another thread.
bool g_scan_nt = true;  // EDV_SCAN_NT=0: ordinary stores (A/B); set per scan call
inline void nt_slot96(char* dst, const unsigned char* text, size_t n) {  // dst 16-byte aligned, n <= 95
  alignas(16) char b[96];
  memcpy(b, text, n);
  memset(b + n, 0, 95 - n);
  b[95] = (char)n;
  for (int k = 0; k < 6; ++k) _mm_stream_si128((__m128i*)(dst + 16 * k), _mm_load_si128((const __m128i*)(b + 16 * k)));
}
inline void nt_copy(char* dst, const char* src, size_t n) {
  const size_t head = (size_t)((16 - ((uintptr_t)dst & 15)) & 15);
  if (n < head + 32) {
    memcpy(dst, src, n);
    return;
  }
  memcpy(dst, src, head);
  dst += head, src += head, n -= head;
  for (; n >= 16; dst += 16, src += 16, n -= 16) _mm_stream_si128((__m128i*)dst, _mm_loadu_si128((const __m128i*)src));
  memcpy(dst, src, n);
}

struct ScanItem {
  PyObject* m = nullptr;
  const unsigned char* sp = nullptr;
  Py_ssize_t ns = 0;
  uint32_t uid = 0xffffffffu;
  uint8_t state = 0;  // 0 Python path, 1 fast, 2 serialization deferred
  uint8_t text = 0;   // slot mode: the signature's base58 text goes to the GPU (decodes to 64 bytes)
  uint16_t buf = 0;   // which buffer holds its decoded signature / serialization
  uint32_t sig_len = 0, ser_len = 0;
  uint64_t sig_at = 0, ser_at = 0;
};
struct alignas(64) ScanBuf {  // one cache line per worker: the string headers change on every append
  std::string sig;
  OutBuf ser;
};

// CPUs this process may use: its affinity mask, capped by a cgroup v2 CPU quota
// (cpu.max "quota period"; the GPU box shows 256 CPUs but grants 16 of them).
int cpu_budget() {
  static const int budget = [] {
    cpu_set_t set;
    int aff = sched_getaffinity(0, sizeof set, &set) == 0 ? CPU_COUNT(&set) : 0;
    if (aff <= 0) aff = (int)std::max(1u, std::thread::hardware_concurrency());
    int quota = aff;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long period = 0;
      if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
        quota = (int)std::max(1L, atol(q) / period);
      fclose(f);
    }
    return std::max(1, std::min(aff, quota));
  }();
  return budget;
}

// Scan workers for n items: one per 2k items (two kScanChunk chunks or more each), up to the
// CPUs this process may use and at most kMaxScanThreads (a node host with more CPUs than the GPU
// box's 16-CPU share scans a large batch on more of them).
constexpr int kMaxScanThreads = 48;
int scan_threads(Py_ssize_t n, int want) {
  if (want > 0) return std::min(want, 64);
  const char* env = getenv("EDV_SCAN_THREADS");  // at most this many workers (A/B)
  const int env_max = env ? atoi(env) : 0;
  const Py_ssize_t by_size = n / 2048 + 1;
  const Py_ssize_t cap = env_max > 0 ? (Py_ssize_t)env_max : (Py_ssize_t)kMaxScanThreads;
  return (int)std::max<Py_ssize_t>(1, std::min<Py_ssize_t>({(Py_ssize_t)cpu_budget(), cap, by_size}));
}

// Host workers of the scan and the pack: the calling thread (worker 0, left
// where it is) plus t - 1 pool threads (host_pool.h).  EDV_SCAN_PIN=1 pins each helper
// to its own CPU (worker_cpus): a new thread starts next to the thread that
// spawned it and the scheduler spreads short-lived threads only after
// milliseconds, so on a dedicated 8-CPU host 2 and 4 unpinned workers ran no
// faster than 1 and pinned ones 2.0x and 4.1x; on the shared GPU box
// (16-CPU quota out of 256 CPUs) unpinned workers were faster (1M requests end
// to end 17.7-19.7 vs 15.3-16.5 M/s pinned: the scheduler finds idle CPUs), so
// pinning is off by default.  Items go out in chunks of kScanChunk from a
// shared counter, so a worker whose CPU is busy with other work takes fewer.
// f(worker, begin, end) per chunk.
constexpr Py_ssize_t kScanChunk = 1024;

// Software prefetch of the requests ahead of the worker (on unless EDV_SCAN_PREFETCH=0): a request is
// ~10 small objects scattered over the heap (each json-decoded on its own), so the scan waits on
// one cache miss after another.  Stages, each reading only what an earlier stage fetched: the
// dict of item i + 10; its key table (i + 7); its keys and values (i + 4); the key tables of
// dict values (i + 2); their keys and values (i + 1).  Key-table entries are walked directly
// on CPython 3.10's combined-table layout (elsewhere nothing past the dict is prefetched).
inline void pf(const void* p) { __builtin_prefetch(p); }
inline void pf_lines(const void* p, int n) {
  for (int k = 0; k < n; ++k) __builtin_prefetch((const char*)p + 64 * k);
}
// (K scales every distance: EDV_SCAN_PF=2 or 3 prefetches two or three times as far ahead, A/B)
template <int K = 1>
inline void prefetch_ahead(PyObject** items, Py_ssize_t i, Py_ssize_t b) {
  if (i + 10 * K < b) pf(items[i + 10 * K]);
  if (i + 7 * K < b) {
    PyObject* o = items[i + 7 * K];
    if (Py_TYPE(o) == &PyDict_Type) pf_lines(((PyDictObject*)o)->ma_keys, 3);
  }
#ifdef EDV_HAVE_DK
  Py_ssize_t n;
  if (i + 4 * K < b)
    if (const DkEntry* e = dk_entries(items[i + 4 * K], n))
      for (Py_ssize_t j = 0; j < n; ++j)
        if (e[j].v) {
          pf(e[j].k);
          pf_lines(e[j].v, 2);
        }
  if (i + 2 * K < b)
    if (const DkEntry* e = dk_entries(items[i + 2 * K], n))
      for (Py_ssize_t j = 0; j < n; ++j)
        if (e[j].v && Py_TYPE(e[j].v) == &PyDict_Type) pf_lines(((PyDictObject*)e[j].v)->ma_keys, 3);
  if (i + K < b)
    if (const DkEntry* e = dk_entries(items[i + K], n))
      for (Py_ssize_t j = 0; j < n; ++j) {
        Py_ssize_t n2;
        if (e[j].v)
          if (const DkEntry* e2 = dk_entries(e[j].v, n2))
            for (Py_ssize_t q = 0; q < n2; ++q)
              if (e2[q].v) {
                pf(e2[q].k);
                pf_lines(e2[q].v, 2);
              }
      }
#endif
}

// f(worker, begin, end) per chunk of kScanChunk items, chunks taken from a
// shared counter by the caller and t - 1 pool helpers, so a worker whose CPU
// is busy with other work takes fewer.
template <class F>
void run_chunks(Py_ssize_t n, int t, F&& f, Py_ssize_t chunk = kScanChunk) {
  if (t <= 1 || n <= chunk) {
    // serially, but still chunk by chunk: callers may key per-chunk state on a / chunk (the staged
    // scan publishes one slot_done flag per kStageChunk)
    for (Py_ssize_t a = 0; a < n; a += chunk) f(0, a, std::min(n, a + chunk));
    return;
  }
  std::atomic<Py_ssize_t> next{0};
  const std::function<void(int)> body = [&](int w) {
    for (;;) {
      const Py_ssize_t a = next.fetch_add(chunk, std::memory_order_relaxed);
      if (a >= n) break;
      f(w, a, std::min(n, a + chunk));
    }
  };
  HostPool::get().run(t, body);
}

// EDV_SCAN_NUMA=1 (A/B): the scan's helper threads run on the CPUs of the NUMA node that holds
// the batch's request objects (the node of the pages of three sampled dicts, get_mempolicy), so a
// batch built on another node than the helpers happened to run on is not walked across the
// socket link.  The calling thread is left where it is.  Measured slower on the GPU box (2 x EPYC
// 9575F, NPS1, a 16-CPU quota over 256 CPUs): 39.0-48.5 against 49.1-50.6 M/s whole node
// (profiles/r10y) -- off by default.
inline int numa_node_cpus(int node, cpu_set_t& set) {
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  char buf[4096];
  const size_t len = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[len] = 0;
  CPU_ZERO(&set);
  int count = 0;
  for (char* p = buf; *p && *p != '\n';) {
    char* end;
    long a = strtol(p, &end, 10), b = a;
    if (end == p) break;
    if (*end == '-') b = strtol(end + 1, &end, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c, ++count) CPU_SET((int)c, &set);
    p = *end == ',' ? end + 1 : end;
  }
  return count;
}
inline void numa_follow(PyObject** items, Py_ssize_t n) {
  static const bool on = getenv("EDV_SCAN_NUMA") && getenv("EDV_SCAN_NUMA")[0] == '1';
  if (!on) return;
  int votes[4] = {-1, -1, -1, -1};
  const Py_ssize_t at[3] = {0, n / 2, n - 1};
  for (int k = 0; k < 3; ++k) {
    int node = -1;
    // MPOL_F_NODE | MPOL_F_ADDR: the node of the page holding the address
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, (void*)items[at[k]], 3UL) == 0) votes[k] = node;
  }
  const int node = votes[0] >= 0 && (votes[0] == votes[1] || votes[0] == votes[2]) ? votes[0]
                   : votes[1] >= 0 && votes[1] == votes[2]                      ? votes[1]
                                                                                  : votes[0];
  if (node < 0) return;
  cpu_set_t set, mine;
  if (numa_node_cpus(node, set) <= 0 || sched_getaffinity(0, sizeof mine, &mine) != 0) return;
  CPU_AND(&set, &set, &mine);
  if (CPU_COUNT(&set) == 0) return;
  HostPool& pool = HostPool::get();
  if (!pool.same_affinity(set)) pool.set_affinity(set);
}

// Scratch kept across calls.  A fresh 1M-request batch would otherwise touch
// ~600 MB of newly mapped memory per call (page faults on first touch, unmaps
// on free), which measured ~25 % of the scan.  The scan holds the GIL from
// start to end, so calls never overlap.
struct ScanScratch {
  std::vector<ScanItem> it;
  std::vector<PyObject*> idr_of;
  std::vector<ScanBuf> bufs;
  std::vector<uint64_t> off;
  std::string fast, shortv;
  std::vector<uint32_t> uidx;
  std::vector<uint64_t> spans;  // staged mode: message starts [n] then ends [n]
};

// Staged mode (defer = 2): edverify.h edv_stage_put, called by the workers.
using StageFn = int (*)(void*, const void*, uint64_t, uint64_t);
// edverify.h edv_verify_staged_part, called by the staged scan's copier thread
using PartFn = int (*)(void*, const void*, uint64_t, uint64_t, const uint64_t*, uint64_t, uint64_t, uint64_t);
constexpr Py_ssize_t kStageChunk = 4096;  // items per staged chunk: ~0.8 MB of messages, 0.4 MB of slots

// The copies of a staged scan, issued by one thread of their own so no worker ever waits on the
// runtime: workers publish each finished chunk (its message reservation, by reservation order,
// and its slot range, by chunk index); the copier advances over the contiguous done prefix of
// each and queues one edv_stage_put per >= kCopyGrain bytes (and the remainder at the end).
constexpr uint64_t kCopyGrain = 4ull << 20;
constexpr int kSeqShift = 44;  // message cursor: reservation number << 44 | byte position
struct StageCopier {
  StageFn fn = nullptr;
  void* ctx = nullptr;
  const char* smsg = nullptr;
  const char* dsig = nullptr;
  uint64_t slot_base = 0, slot_bytes_per_chunk = 0, slot_bytes_total = 0;
  size_t nchunks = 0;
  std::unique_ptr<std::atomic<uint64_t>[]> res_end;  // by reservation number: end byte + 1 once written (0 = not yet)
  std::unique_ptr<std::atomic<uint8_t>[]> slot_done;  // by chunk index
  std::atomic<bool> finished{false};
  std::atomic<bool> failed{false};
  std::thread th;
  uint64_t msg_sent = 0, msg_ready = 0;
  size_t next_res = 0, next_chunk = 0, slot_sent_chunk = 0;
  // parts (edv_verify_staged_part): every part_items items, once their chunks are written and
  // copied, their key ids and spans copied and their kernels queued -- while the scan goes on
  PartFn part_fn = nullptr;
  void* part_ctx = nullptr;
  const void* part_keys = nullptr;
  const uint64_t* part_spans = nullptr;
  uint64_t n_items = 0, part_items = 0, next_part = 0;
  std::atomic<bool> part_failed{false};
  std::unique_ptr<std::atomic<uint32_t>[]> chunk_seq;  // by chunk index: its message reservation number

  void put(const char* src, uint64_t nbytes, uint64_t off) {
#ifdef EDV_STAGE_NODMA  // diagnostic builds only (tools/: the scan's cost without the copies under it)
    return;
#endif
    if (nbytes && fn(ctx, src, nbytes, off) != 0) failed = true;
  }
  void send_ready() {  // every ready message byte and slot, whatever the grain
    if (msg_ready > msg_sent) {
      put(smsg + msg_sent, msg_ready - msg_sent, msg_sent);
      msg_sent = msg_ready;
    }
    const uint64_t s0 = slot_sent_chunk * slot_bytes_per_chunk;
    const uint64_t s1 = std::min<uint64_t>(next_chunk * slot_bytes_per_chunk, slot_bytes_total);
    if (s1 > s0) {
      put(dsig + s0, s1 - s0, slot_base + s0);
      slot_sent_chunk = next_chunk;
    }
  }
  // the parts whose chunks are all written (slot_done) and whose messages are in the ready prefix
  void launch_parts() {
    if (!part_fn || part_failed) return;
    while (next_part * part_items < n_items) {
      const uint64_t lo = next_part * part_items, hi = std::min(n_items, lo + part_items);
      const size_t c0 = (size_t)(lo / kStageChunk), c1 = (size_t)((hi + kStageChunk - 1) / kStageChunk);
      if (c1 > next_chunk) return;  // (next_chunk: the contiguous prefix of written chunks)
      for (size_t c = c0; c < c1; ++c)
        if (chunk_seq[c].load(std::memory_order_acquire) >= next_res) return;
      send_ready();
      if (part_fn(part_ctx, part_keys, slot_base, 0, part_spans, n_items, lo, hi) != 0) {
        part_failed = true;
        return;
      }
      ++next_part;
    }
  }
  // one pass over what became ready; `flush` sends every ready byte
  void pump(bool flush) {
    while (next_res < nchunks) {
      const uint64_t e = res_end[next_res].load(std::memory_order_acquire);
      if (!e) break;
      msg_ready = e - 1;
      ++next_res;
    }
    if (msg_ready > msg_sent && (flush || msg_ready - msg_sent >= kCopyGrain)) {
      put(smsg + msg_sent, msg_ready - msg_sent, msg_sent);
      msg_sent = msg_ready;
    }
    while (next_chunk < nchunks && slot_done[next_chunk].load(std::memory_order_acquire)) ++next_chunk;
    const uint64_t s0 = slot_sent_chunk * slot_bytes_per_chunk;
    const uint64_t s1 = std::min<uint64_t>(next_chunk * slot_bytes_per_chunk, slot_bytes_total);
    if (s1 > s0 && (flush || s1 - s0 >= kCopyGrain)) {
      put(dsig + s0, s1 - s0, slot_base + s0);
      slot_sent_chunk = next_chunk;
    }
    launch_parts();
  }
  void start() {
    th = std::thread([this] {
      while (!finished.load(std::memory_order_acquire)) {
        pump(false);
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    });
  }
  void finish() {  // after every worker is done: join, then send the rest
    finished = true;
    if (th.joinable()) th.join();
    pump(true);
  }
  ~StageCopier() {
    finished = true;
    if (th.joinable()) th.join();
  }
};
// One spare scratch kept across calls (taken by a scan, given back when it --
// or the pack handle of a deferred scan -- is done); a scan entered while the
// spare is out (a garbage collection's finalizer inside a scan, a second
// deferred batch) gets a fresh one.  Touched only under the GIL.
ScanScratch* g_spare = nullptr;
ScanScratch* take_scratch() {
  ScanScratch* s = g_spare ? g_spare : new ScanScratch;
  g_spare = nullptr;
  return s;
}
void give_scratch(ScanScratch* s) {
  if (!s) return;
  if (!g_spare)
    g_spare = s;
  else
    delete s;
}

// A deferred scan's state for pack_range: the scratch (items, worker buffers,
// offsets), the output pointers and references to the output objects.
struct PackState {
  ScanScratch* S = nullptr;
  PyObject *o_sig = nullptr, *o_msg = nullptr;
  char *dsig = nullptr, *dmsg = nullptr;
  int sig_slot = 64, t = 1;
  Py_ssize_t n = 0;
};
void pack_items(const PackState& P, Py_ssize_t lo, Py_ssize_t hi);
void pack_capsule_free(PyObject* cap) {
  PackState* P = (PackState*)PyCapsule_GetPointer(cap, "edv.pack");
  if (!P) return;
  give_scratch(P->S);
  Py_XDECREF(P->o_sig);
  Py_XDECREF(P->o_msg);
  delete P;
}

// Output buffer for (5): the caller's bytearray grown to `need` bytes (never
// shrunk, so its pages stay mapped from call to call); or any other writable
// C-contiguous buffer of at least `need` bytes -- the authenticator passes the
// engine's pinned host memory (edv_host_alloc), so the GPU call copies from it
// without staging; or a fresh bytes object when neither fits (a bytearray with
// a live export, a buffer that is too small).  The object is returned as the
// result and the pointer stays valid while the caller holds it.
PyObject* out_buffer(PyObject* ba, Py_ssize_t need, char** data) {
  if (ba && PyByteArray_CheckExact(ba)) {
    if (PyByteArray_GET_SIZE(ba) >= need || PyByteArray_Resize(ba, need) == 0) {
      Py_INCREF(ba);
      *data = PyByteArray_AS_STRING(ba);
      return ba;
    }
    PyErr_Clear();
  } else if (ba && ba != Py_None && PyObject_CheckBuffer(ba)) {
    Py_buffer view;
    if (PyObject_GetBuffer(ba, &view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) == 0) {
      const bool fits = view.len >= need;
      char* p = (char*)view.buf;
      // a buffer with a memory owner outside Python (ctypes over pinned host memory): the
      // caller keeps the owner alive while it uses the result
      PyBuffer_Release(&view);
      if (fits) {
        Py_INCREF(ba);
        *data = p;
        return ba;
      }
    } else {
      PyErr_Clear();
    }
  }
  PyObject* b = PyBytes_FromStringAndSize(nullptr, need);
  if (b) *data = PyBytes_AS_STRING(b);
  return b;
}

// Owned references released on every exit, an exception's unwinding included.
struct PyRefs {
  PyObject* fm = nullptr;
  PyObject* ign = nullptr;
  PyObject* o_sig = nullptr;
  PyObject* o_msg = nullptr;
  ~PyRefs() {
    Py_XDECREF(o_sig);
    Py_XDECREF(o_msg);
    Py_XDECREF(fm);
    Py_XDECREF(ign);
  }
};

PyObject* scan_impl_body(PyObject* args, bool unique_form, PyRefs& refs) {
  PyObject *msgs, *ignore = Py_None, *out = Py_None, *stager = Py_None, *spec = Py_None;
  int want_threads = 0, sig_slot = 64, defer = 0;
  unsigned long long slot_base = 0;
  if (!PyArg_ParseTuple(args, "O|OiOiiOKO", &msgs, &ignore, &want_threads, &out, &sig_slot, &defer, &stager,
                        &slot_base, &spec))
    return nullptr;
  if (defer && !unique_form) {
    PyErr_SetString(PyExc_ValueError, "defer needs scan_batch_u");
    return nullptr;
  }
  // staged mode: (edv_stage_put address, context address); messages at staging offset 0, slots
  // at slot_base; both output buffers must be the engine's pinned memory
  const bool staged = defer == 2;
  StageFn stage_fn = nullptr;
  void* stage_ctx = nullptr;
  if (staged) {
    unsigned long long fa = 0, ca = 0;
    if (!PyTuple_Check(stager) || !PyArg_ParseTuple(stager, "KK", &fa, &ca) || !fa || !ca) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "staged scan: stager = (edv_stage_put, ctx)");
      return nullptr;
    }
    stage_fn = (StageFn)(uintptr_t)fa;
    stage_ctx = (void*)(uintptr_t)ca;
    if (sig_slot != kSigSlot) {
      PyErr_SetString(PyExc_ValueError, "staged scan needs signature slots");
      return nullptr;
    }
  }
  if (sig_slot != 64 && sig_slot != kSigSlot) {
    PyErr_Format(PyExc_ValueError, "slot must be 64 (raw signatures) or %d (base58 slots)", kSigSlot);
    return nullptr;
  }
  const bool slots = sig_slot == kSigSlot;
  // staged mode with speculation: spec = (kid_map, key-id buffer (4 n bytes, the engine's pinned
  // memory), (edv_verify_staged_part address, context address), items per part): each request's
  // key id from the map by its identifier (0xffffffff: not in it) written while scanning, and each
  // part's kernels queued by the copier as soon as the part is staged
  const KidMap* kmap = nullptr;
  uint32_t* kid_out = nullptr;
  PartFn part_fn = nullptr;
  void* part_ctx = nullptr;
  unsigned long long part_items = 0;
  if (spec != Py_None) {
    PyObject *cap, *kbuf, *pf;
    unsigned long long fa = 0, ca = 0;
    if (!staged || !PyTuple_Check(spec) || !PyArg_ParseTuple(spec, "OOOK", &cap, &kbuf, &pf, &part_items) ||
        !PyTuple_Check(pf) || !PyArg_ParseTuple(pf, "KK", &fa, &ca) || !fa || !ca || !part_items ||
        part_items % kStageChunk) {
      if (!PyErr_Occurred())
        PyErr_SetString(PyExc_ValueError, "spec = (kid_map, pinned key ids, (part fn, ctx), items per part: k * 4096)");
      return nullptr;
    }
    kmap = (const KidMap*)PyCapsule_GetPointer(cap, "edv.kidmap");
    if (!kmap) return nullptr;
    Py_buffer view;
    if (PyObject_GetBuffer(kbuf, &view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) return nullptr;
    const bool fits = (uint64_t)view.len >= 4 * (uint64_t)PySequence_Size(msgs);
    kid_out = (uint32_t*)view.buf;
    PyBuffer_Release(&view);  // the caller keeps the owner alive
    if (!fits) {
      PyErr_SetString(PyExc_ValueError, "spec: the key-id buffer holds fewer than 4 n bytes");
      return nullptr;
    }
    part_fn = (PartFn)(uintptr_t)fa;
    part_ctx = (void*)(uintptr_t)ca;
  }
  PyObject *out_sig = nullptr, *out_msg = nullptr, *out_spans = nullptr;
  if (out != Py_None) {
    if (!PyList_CheckExact(out) || PyList_GET_SIZE(out) < 2 || PyList_GET_SIZE(out) > 3) {
      PyErr_SetString(PyExc_TypeError,
                      "out must be a list of two (or, staged, three) writable buffers (bytearray, pinned memory)");
      return nullptr;
    }
    out_sig = PyList_GET_ITEM(out, 0);
    out_msg = PyList_GET_ITEM(out, 1);
    if (PyList_GET_SIZE(out) == 3) out_spans = PyList_GET_ITEM(out, 2);
  }
  PyObject* fm = refs.fm = PySequence_Fast(msgs, "msgs must be a sequence");
  if (!fm) return nullptr;
  PyObject* ign = nullptr;
  if (ignore != Py_None) {
    ign = refs.ign = PySequence_Fast(ignore, "ignore must be a sequence");
    if (!ign) return nullptr;
  }
  static PyObject* k_sig = PyUnicode_InternFromString("signature");
  static PyObject* k_idr = PyUnicode_InternFromString("identifier");
  PyObject* const top_keys[2] = {k_sig, k_idr};
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fm);
  struct Held {  // the scratch goes back to the spare slot on every exit unless a pack handle takes it
    ScanScratch* s = take_scratch();
    ~Held() { give_scratch(s); }
  } held;
  ScanScratch& S = *held.s;
  std::vector<ScanItem>& it = S.it;
  std::vector<PyObject*>& idr_of = S.idr_of;  // borrowed (the dicts hold them)
  it.resize((size_t)n);                       // entries reset by the workers
  idr_of.resize((size_t)n);
  const bool prof = getenv("EDV_SCAN_PROFILE") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto t_start = now();
  PyObject** items = PySequence_Fast_ITEMS(fm);
  // (1) on the workers, per item: the checks of authenticate():72-91 (fields
  // found by PyDict_Next: a dict with a key that is not an exact str takes the
  // Python path), base58 decode, serialization, and the identifier's slot in
  // the worker's own table of distinct identifiers
  const int t = scan_threads(n, want_threads);
  if (t > 1 && n > 0) numa_follow(items, n);
  std::vector<ScanBuf>& bufs = S.bufs;  // bufs[t]: items redone under the GIL
  if (bufs.size() < (size_t)t + 1) bufs.resize((size_t)t + 1);
  for (ScanBuf& b : bufs) {
    b.sig.clear();
    b.ser.clear();
  }
  struct alignas(64) WorkerIdrs {  // a cache line (or more) of its own per worker
    IdrTable slot;
    std::vector<PyObject*> obj;
    std::vector<uint32_t> kid;      // speculation: the key id of each of its identifiers (kmap)
    std::vector<Py_ssize_t> first;  // the item where the worker met it first
    std::vector<uint64_t> hash;     // IdrTable::hash of each of its identifiers (the merge's partitions)
    std::vector<char> txt;          // the first IdrTable::kInl bytes of each (the merge compares these)
    std::vector<uint32_t> tlen;     // and its length
    size_t deferred = 0;            // items left for the GIL pass (3)
#ifdef EDV_HAVE_DK
    std::unique_ptr<ShapeCache> shapes;  // this call's remembered dict shapes (shaped_dict)
#endif
  };
  std::vector<WorkerIdrs> tabs((size_t)t);
  // remembered dict shapes (shaped_dict); EDV_SCAN_SHAPES=0: wser_dict for every request (A/B)
  const char* shape_env = getenv("EDV_SCAN_SHAPES");
  const bool shapes = g_scan_direct_env() && !(shape_env && shape_env[0] == '0');
  for (WorkerIdrs& w : tabs) {
    w.slot.reset(1024);
#ifdef EDV_HAVE_DK
    if (shapes) w.shapes.reset(new ShapeCache);
#endif
  }
  // the signature output (n slots) is sized before the scan: in slot mode the workers write an
  // item's base58 text slot while its text is still in cache (phase 5 writes the rest)
  char* dsig = nullptr;
  PyObject* o_sig = refs.o_sig = out_buffer(out_sig, (Py_ssize_t)n * sig_slot, &dsig);
  if (!o_sig) return nullptr;
  // staged mode: the message buffer is the caller's pinned buffer, filled by a bump cursor chunk
  // by chunk (each chunk's bytes contiguous, chunks in completion order; item spans say where)
  char* smsg = nullptr;
  uint64_t smsg_cap = 0;
  uint64_t* spans_p = nullptr;  // staged: starts [n] then ends [n]
  std::atomic<uint64_t> scursor{0};
  std::atomic<bool> staged_ok{true};
  StageCopier copier;
  if (staged) {
    Py_buffer view;
    if (!out_msg || PyObject_GetBuffer(out_msg, &view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) {
      PyErr_Clear();
      PyErr_SetString(PyExc_ValueError, "staged scan: out[1] must be a writable buffer");
      return nullptr;
    }
    smsg = (char*)view.buf;
    smsg_cap = (uint64_t)view.len;
    PyBuffer_Release(&view);  // the caller keeps the owner alive
    // the item spans go straight into out[2] when it holds 16 n bytes (the engine's pinned memory:
    // edv_verify_staged then DMAs them with no copy), else into the scratch and a bytes result
    spans_p = nullptr;
    if (out_spans && out_spans != Py_None) {
      if (PyObject_GetBuffer(out_spans, &view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) == 0) {
        if ((uint64_t)view.len >= 16 * (uint64_t)n) spans_p = (uint64_t*)view.buf;
        PyBuffer_Release(&view);
      } else {
        PyErr_Clear();
      }
    }
    if (!spans_p) {
      S.spans.resize(2 * (size_t)n);
      spans_p = S.spans.data();
    }
  }
  std::vector<std::vector<uint8_t>> sigs((size_t)t);
  for (int w = 0; w < t; ++w) {  // no-ops once a batch of this size has been seen
    bufs[(size_t)w].sig.reserve((size_t)(n / t + kScanChunk) * 64);
    bufs[(size_t)w].ser.reserve((size_t)(n / t + kScanChunk) * 200);
  }
  // staged mode, at the end of each chunk [a, b) of phase (1): the chunk's messages (crypto_sign_open's
  // sm[64:]) at the bump cursor, the slots the worker has not written (raw signatures, zeroed slots),
  // the item spans, and the two copies queued -- so the DMA runs while the scan goes on
  const auto stage_chunk = [&](int w, Py_ssize_t a, Py_ssize_t b) {
    const ScanBuf& sb = bufs[(size_t)w];
    uint64_t total = 0;
    for (Py_ssize_t i = a; i < b; ++i) {
      const ScanItem& x = it[(size_t)i];
      if (x.state != 1) continue;
      const uint64_t ls = x.sig_len, lm = x.ser_len;
      total += x.text ? lm : (ls + lm >= 64 ? ls + lm - 64 : 0);
    }
    const uint64_t got = scursor.fetch_add(total + (1ull << kSeqShift), std::memory_order_relaxed);
    const size_t seq = (size_t)(got >> kSeqShift);
    const uint64_t pos = got & ((1ull << kSeqShift) - 1);
    if (copier.chunk_seq) copier.chunk_seq[(size_t)(a / kStageChunk)].store((uint32_t)seq, std::memory_order_relaxed);
    if (pos + total > smsg_cap) {
      if (g_scan_nt) _mm_sfence();
      staged_ok = false;  // the buffer was sized from earlier batches: the caller re-scans unstaged
      copier.res_end[seq].store(pos + 1, std::memory_order_release);  // (nothing of it is copied)
      copier.slot_done[(size_t)(a / kStageChunk)].store(1, std::memory_order_release);
      return;
    }
    uint64_t at = pos;
    uint64_t* st0 = spans_p;
    uint64_t* en0 = st0 + n;
    for (Py_ssize_t i = a; i < b; ++i) {
      const ScanItem& x = it[(size_t)i];
      char* ds = dsig + (size_t)i * sig_slot;
      st0[i] = en0[i] = at;
      if (x.state == 1 && x.text) {  // the slot was written in the item loop
        if (g_scan_nt)
          nt_copy(smsg + at, sb.ser.data() + x.ser_at, x.ser_len);
        else
          memcpy(smsg + at, sb.ser.data() + x.ser_at, x.ser_len);
        at += x.ser_len;
        en0[i] = at;
        continue;
      }
      memset(ds + 64, 0, (size_t)sig_slot - 64);  // slot[95] = 0: raw R || S in bytes 0..63
      const uint64_t ls = x.sig_len, lm = x.ser_len;
      if (x.state != 1 || ls + lm < 64) {
        memset(ds, 0, 64);
        continue;
      }
      const char* sr = sb.ser.data() + x.ser_at;
      const char* sg = sb.sig.data() + x.sig_at;
      char* dm = smsg + at;
      if (ls >= 64) {  // sm[64:] = sig[64:] || ser
        memcpy(ds, sg, 64);
        memcpy(dm, sg + 64, ls - 64);
        memcpy(dm + (ls - 64), sr, lm);
      } else {
        memcpy(ds, sg, ls);
        memcpy(ds + ls, sr, 64 - ls);
        memcpy(dm, sr + (64 - ls), lm - (64 - ls));
      }
      at += ls + lm - 64;
      en0[i] = at;
    }
    if (g_scan_nt) _mm_sfence();  // the chunk's non-temporal stores before the copier sees the chunk
    copier.res_end[seq].store(pos + total + 1, std::memory_order_release);
    copier.slot_done[(size_t)(a / kStageChunk)].store(1, std::memory_order_release);
  };
  if (staged) {
    copier.fn = stage_fn;
    copier.ctx = stage_ctx;
    copier.smsg = smsg;
    copier.dsig = dsig;
    copier.slot_base = slot_base;
    copier.slot_bytes_per_chunk = (uint64_t)kStageChunk * sig_slot;
    copier.slot_bytes_total = (uint64_t)n * sig_slot;
    copier.nchunks = (size_t)((n + kStageChunk - 1) / kStageChunk);
    copier.res_end.reset(new std::atomic<uint64_t>[copier.nchunks]);
    copier.slot_done.reset(new std::atomic<uint8_t>[copier.nchunks]);
    if (part_fn) {
      copier.chunk_seq.reset(new std::atomic<uint32_t>[copier.nchunks]);
      copier.part_fn = part_fn;
      copier.part_ctx = part_ctx;
      copier.part_keys = kid_out;
      copier.part_spans = spans_p;
      copier.n_items = (uint64_t)n;
      copier.part_items = part_items;
    }
    for (size_t c = 0; c < copier.nchunks; ++c) {
      copier.res_end[c].store(0, std::memory_order_relaxed);
      copier.slot_done[c].store(0, std::memory_order_relaxed);
    }
    copier.start();
  }
  // software prefetch ahead of the workers (prefetch_ahead): the scan 18.4-19.8 vs 19.7-21.7 ms per
  // 1M on the box's 16 CPUs, alternating in one process (profiles/r05p/scan_ab.log); EDV_SCAN_PREFETCH=0
  // turns it off
  const char* pf_env = getenv("EDV_SCAN_PREFETCH");
  const bool prefetch = !(pf_env && pf_env[0] == '0');
  const char* pfs_env = getenv("EDV_SCAN_PF");  // the distances' scale (A/B): 1 (default), 2, 3
  const int pf_scale = pfs_env ? atoi(pfs_env) : 1;
  const char* dir_env = getenv("EDV_SCAN_DIRECT");
  g_scan_direct = !(dir_env && dir_env[0] == '0');
  // non-temporal stores for what only the DMA reads: the staged scan's slots and messages
  const char* nt_env = getenv("EDV_SCAN_NT");
  g_scan_nt = staged && !(nt_env && nt_env[0] == '0');
  const bool nt_slots = g_scan_nt;
  run_chunks(n, t, [&](int w, Py_ssize_t a, Py_ssize_t b) {
    ScanBuf& sb = bufs[(size_t)w];
    WorkerIdrs& tab = tabs[(size_t)w];
    std::vector<uint8_t>& sig = sigs[(size_t)w];
    for (Py_ssize_t i = a; i < b; ++i) {
      PyObject* m = items[i];
      ScanItem& x = it[(size_t)i];
      x = ScanItem{};
      idr_of[(size_t)i] = nullptr;
      if (kid_out) kid_out[i] = 0xffffffffu;
      if (prefetch) {
        if (pf_scale == 2)
          prefetch_ahead<2>(items, i, b);
        else if (pf_scale == 3)
          prefetch_ahead<3>(items, i, b);
        else
          prefetch_ahead<1>(items, i, b);
      }
      if (!PyDict_CheckExact(m)) continue;
      // one pass over the request's keys: its signing serialization (kept if the item stays on
      // the fast path) and the signature and identifier values
      PyObject* found[2] = {nullptr, nullptr};
      const size_t at = sb.ser.size();
#ifdef EDV_HAVE_DK
      const WRes r = shapes ? shaped_dict(m, 0, ign, sb.ser, top_keys, found, *tab.shapes)
                            : wser_dict(m, 0, ign, sb.ser, top_keys, found);
#else
      const WRes r = wser_dict(m, 0, ign, sb.ser, top_keys, found);
#endif
      PyObject *sv = found[0], *iv = found[1];
      if (!(sv && iv && PyUnicode_CheckExact(sv) && PyUnicode_GET_LENGTH(sv) > 0 && PyUnicode_CheckExact(iv) &&
            PyUnicode_GET_LENGTH(iv) > 0 && PyUnicode_IS_ASCII(sv))) {
        sb.ser.resize(at);
        continue;  // the Python path raises the reference's exception
      }
      x.m = m;
      if (!PyUnicode_IS_ASCII(iv)) {  // its UTF-8 form may need allocating: under the GIL
        sb.ser.resize(at);
        x.state = 2;
        ++tab.deferred;
        continue;
      }
      x.sp = (const unsigned char*)PyUnicode_1BYTE_DATA(sv);
      x.ns = PyUnicode_GET_LENGTH(sv);
      int len64 = 0;
      if (slots) {  // decoded on the GPU when the text decodes to exactly 64 bytes
        len64 = x.ns <= kSigSlot - 1 ? b58_len64(x.sp, (size_t)x.ns) : 0;
        if (len64 < 0) {
          sb.ser.resize(at);
          continue;  // b58decode raises: the Python path (InvalidSignatureFormat)
        }
      }
      if (len64 == 0 && !b58decode_raw(x.sp, (size_t)x.ns, sig)) {
        sb.ser.resize(at);
        continue;
      }
      if (r != kOk) {
        sb.ser.resize(at);
        x.state = r == kDefer ? 2 : 0;
        tab.deferred += r == kDefer;
        continue;
      }
      x.state = 1;
      x.buf = (uint16_t)w;
      x.ser_at = at;
      x.ser_len = (uint32_t)(sb.ser.size() - at);
      if (len64 == 1) {
        x.text = 1;
        x.sig_len = 64;
        char* ds = dsig + (size_t)i * sig_slot;  // slot: the text, zero padding, its length in the last byte
        if (nt_slots && ((uintptr_t)ds & 15) == 0) {
          nt_slot96(ds, x.sp, (size_t)x.ns);
        } else {
          memcpy(ds, x.sp, (size_t)x.ns);
          memset(ds + x.ns, 0, (size_t)sig_slot - 1 - (size_t)x.ns);
          ds[sig_slot - 1] = (char)x.ns;
        }
      } else {
        x.sig_at = sb.sig.size();
        x.sig_len = (uint32_t)sig.size();
        sb.sig.append((const char*)sig.data(), sig.size());
      }
      idr_of[(size_t)i] = iv;
      bool fresh = false;
      const uint64_t ih = IdrTable::hash((const char*)PyUnicode_1BYTE_DATA(iv), (size_t)PyUnicode_GET_LENGTH(iv));
      x.uid = tab.slot.find_or_add_h(ih, (const char*)PyUnicode_1BYTE_DATA(iv), (size_t)PyUnicode_GET_LENGTH(iv),
                                     (uint32_t)tab.obj.size(), fresh);
      if (fresh) {
        tab.obj.push_back(iv);
        tab.first.push_back(i);
        tab.hash.push_back(ih);  // (computed once: the table's probe and the merge's partition)
        {
          const size_t tn = (size_t)PyUnicode_GET_LENGTH(iv), at = tab.txt.size();
          tab.txt.resize(at + IdrTable::kInl);
          memcpy(tab.txt.data() + at, PyUnicode_1BYTE_DATA(iv), tn < IdrTable::kInl ? tn : IdrTable::kInl);
          tab.tlen.push_back((uint32_t)tn);
        }
        if (kmap) tab.kid.push_back(kmap->get((const char*)PyUnicode_1BYTE_DATA(iv), (size_t)PyUnicode_GET_LENGTH(iv)));
      }
      if (kid_out) kid_out[i] = tab.kid[x.uid];
    }
    if (staged) stage_chunk(w, a, b);
  }, staged ? kStageChunk : kScanChunk);
  if (staged) {
    copier.finish();
    if (copier.failed) staged_ok = false;
  }
  auto t_p1 = now();
  auto t_m1 = t_p1, t_m2 = t_p1;  // (the merge's partition pass / ordering / remap, EDV_SCAN_PROFILE)
  // (2) the workers' identifier tables merged into the batch's, in order of
  // first occurrence in the batch (the single-thread order, whichever worker
  // took which chunk)
  std::vector<PyObject*> uniq;
  std::vector<uint32_t> spec_u;  // speculation: the key id the scan wrote for each distinct identifier
  IdrTable slot;
  slot.reset(tabs.empty() ? 64 : tabs[0].obj.size() + 64);
  std::vector<std::vector<uint32_t>> to_global((size_t)t);
  size_t deferred = 0;
  for (const WorkerIdrs& w : tabs) deferred += w.deferred;
  {
    // partitioned by identifier hash, one partition per worker, merged side by side: each
    // partition keeps its identifiers' earliest first occurrence (every worker's table holds most
    // of a batch's identifiers, so a serial merge compared ~t x distinct texts on one thread); then
    // the distinct identifiers are numbered in order of first occurrence
    size_t ncand = 0;
    for (const WorkerIdrs& w : tabs) ncand += w.obj.size();
    const int P = ncand >= 8192 ? t : 1;  // (a small batch merges on this thread: no helper wake-ups)
    // an identifier's partition from its hash's high half by a multiply (h % P was a 64-bit division
    // per worker entry per partition: ~1.6 ms of a churning batch's merge); the low bits index the tables
    const auto part_of = [P](uint64_t h) -> Py_ssize_t { return (Py_ssize_t)(((h >> 32) * (uint64_t)P) >> 32); };
    struct Part {
      IdrTable tab;
      std::vector<PyObject*> obj;
      std::vector<Py_ssize_t> first;
      std::vector<uint32_t> kid;
      std::vector<uint32_t> gid;
    };
    std::vector<Part> parts((size_t)P);
    for (int w = 0; w < t; ++w) to_global[(size_t)w].resize(tabs[(size_t)w].obj.size());
    run_chunks(P, P, [&](int, Py_ssize_t a, Py_ssize_t b) {
      for (Py_ssize_t p = a; p < b; ++p) {
        Part& pt = parts[(size_t)p];  // (P = 1: the one partition, serially)
        pt.tab.reset(tabs.empty() ? 64 : tabs[0].obj.size() / (size_t)P + 64);
        for (int w = 0; w < t; ++w) {
          const WorkerIdrs& tb = tabs[(size_t)w];
          for (size_t u = 0; u < tb.obj.size(); ++u) {
            const uint64_t h = tb.hash[u];
            if (part_of(h) != p) continue;
            PyObject* o = tb.obj[u];
            bool fresh = false;
            // the worker's copy of the text when it is short (no cache miss on the object), else its data
            const bool copied = tb.tlen.size() > u;
            const size_t on = copied ? (size_t)tb.tlen[u] : (size_t)PyUnicode_GET_LENGTH(o);
            const char* op = copied && on <= IdrTable::kInl
                                 ? tb.txt.data() + u * IdrTable::kInl
                                 : (const char*)PyUnicode_1BYTE_DATA(o);
            const uint32_t l = pt.tab.find_or_add_h(h, op, on, (uint32_t)pt.obj.size(), fresh);
            if (fresh) {
              pt.obj.push_back(o);
              pt.first.push_back(tb.first[u]);
              if (kmap) pt.kid.push_back(tb.kid[u]);  // (the map's id for this text: the same in every worker)
            } else if (tb.first[u] < pt.first[l]) {
              pt.first[l] = tb.first[u];
              pt.obj[l] = o;  // the object of its first occurrence, as a serial scan returns it
            }
            to_global[(size_t)w][u] = l;  // partition-local for now
          }
        }
      }
    }, 1);
    t_m1 = now();
    struct Cand {
      Py_ssize_t first;
      int p;
      uint32_t local;
    };
    size_t ncand_u = 0;
    for (int p = 0; p < P; ++p) ncand_u += parts[(size_t)p].obj.size();
    if (P > 1 && ncand_u > 4096) {
      // many distinct identifiers (a churning batch: ~30k of 250k items), ordered on the workers: the
      // batch's positions cut into P ranges, worker r takes from every partition the identifiers
      // first met in range r and sorts them; a prefix sum over the ranges' counts gives each its
      // global number.  (Ordered on one thread -- a comparison sort, a position bitmap or a radix
      // sort alike -- it took ~2 ms: the partitions' arrays were written by the other cores.)
      uniq.resize(ncand_u);
      if (kmap) spec_u.resize(ncand_u);
      std::vector<std::vector<Cand>> by_range((size_t)P);
      std::vector<size_t> base((size_t)P + 1, 0);
      const auto range_of = [n, P](Py_ssize_t f) { return (int)((uint64_t)f * (uint64_t)P / (uint64_t)n); };
      run_chunks(P, P, [&](int, Py_ssize_t ra, Py_ssize_t rb) {
        for (Py_ssize_t r = ra; r < rb; ++r) {
          std::vector<Cand>& mine = by_range[(size_t)r];
          for (int p = 0; p < P; ++p) {
            const Part& pt = parts[(size_t)p];
            for (size_t l = 0; l < pt.first.size(); ++l)
              if (range_of(pt.first[l]) == (int)r) mine.push_back(Cand{pt.first[l], p, (uint32_t)l});
          }
          std::sort(mine.begin(), mine.end(), [](const Cand& x, const Cand& y) { return x.first < y.first; });
        }
      }, 1);
      for (int r = 0; r < P; ++r) base[(size_t)r + 1] = base[(size_t)r] + by_range[(size_t)r].size();
      for (int p = 0; p < P; ++p) parts[(size_t)p].gid.resize(parts[(size_t)p].obj.size());
      run_chunks(P, P, [&](int, Py_ssize_t ra, Py_ssize_t rb) {
        for (Py_ssize_t r = ra; r < rb; ++r) {
          size_t g = base[(size_t)r];
          for (const Cand& c : by_range[(size_t)r]) {
            Part& pt = parts[(size_t)c.p];
            pt.gid[c.local] = (uint32_t)g;
            uniq[g] = pt.obj[c.local];
            if (kmap) spec_u[g] = pt.kid[c.local];
            ++g;
          }
        }
      }, 1);
    } else {
      std::vector<Cand> cand;
      for (int p = 0; p < P; ++p) {
        Part& pt = parts[(size_t)p];
        pt.gid.resize(pt.obj.size());
        for (size_t l = 0; l < pt.obj.size(); ++l) cand.push_back(Cand{pt.first[l], p, (uint32_t)l});
      }
      std::sort(cand.begin(), cand.end(), [](const Cand& x, const Cand& y) { return x.first < y.first; });
      uniq.reserve(cand.size());
      for (const Cand& c : cand) {
        Part& pt = parts[(size_t)c.p];
        pt.gid[c.local] = (uint32_t)uniq.size();
        uniq.push_back(pt.obj[c.local]);
        if (kmap) spec_u.push_back(pt.kid[c.local]);
      }
    }
    t_m2 = now();
    run_chunks(t, P > 1 ? t : 1, [&](int, Py_ssize_t a, Py_ssize_t b) {  // each worker's table, side by side
      for (Py_ssize_t w = a; w < b; ++w) {
        const WorkerIdrs& tb = tabs[(size_t)w];
        std::vector<uint32_t>& tg = to_global[(size_t)w];
        for (size_t u = 0; u < tg.size(); ++u) tg[u] = parts[(size_t)part_of(tb.hash[u])].gid[tg[u]];
      }
    }, 1);
    // the GIL pass (3) below adds the deferred items' identifiers to this table
    for (size_t g = 0; deferred && g < uniq.size(); ++g) {
      bool fresh = false;
      slot.find_or_add((const char*)PyUnicode_1BYTE_DATA(uniq[g]), (size_t)PyUnicode_GET_LENGTH(uniq[g]),
                       (uint32_t)g, fresh);
    }
  }
  // (the items' worker-local ids are mapped in (4), on the workers)
  auto t_p2 = now();
  // (3) the items the workers left (non-ASCII identifiers, floats / big ints /
  // wide-kind keys in the payload), redone under the GIL; none in the steady
  // state, which then skips this pass over the batch
  if (deferred && staged) staged_ok = false;  // rare items redone under the GIL: the caller re-scans unstaged
  if (deferred && !staged) {
    ScanBuf& sb = bufs[(size_t)t];
    std::vector<uint8_t> sig;
    for (Py_ssize_t i = 0; i < n; ++i) {
      ScanItem& x = it[(size_t)i];
      if (x.state != 2) continue;
      x.state = 0;
      PyObject* m = x.m;
      PyObject* sv = PyDict_GetItemWithError(m, k_sig);
      PyObject* iv = sv ? PyDict_GetItemWithError(m, k_idr) : nullptr;
      if (PyErr_Occurred()) PyErr_Clear();
      if (!(sv && iv && PyUnicode_CheckExact(sv) && PyUnicode_GET_LENGTH(sv) > 0 && PyUnicode_CheckExact(iv) &&
            PyUnicode_GET_LENGTH(iv) > 0 && PyUnicode_IS_ASCII(sv)))
        continue;
      Py_ssize_t ni = 0;
      const char* ip = PyUnicode_AsUTF8AndSize(iv, &ni);
      if (!ip) {
        PyErr_Clear();
        continue;
      }
      if (!b58decode_raw((const unsigned char*)PyUnicode_1BYTE_DATA(sv), (size_t)PyUnicode_GET_LENGTH(sv), sig))
        continue;
      const size_t at = sb.ser.size();
      if (!ser_obj(m, 0, ign, sb.ser)) {
        sb.ser.resize(at);
        continue;
      }
      x.state = 1;
      x.buf = (uint16_t)t;
      x.ser_at = at;
      x.ser_len = (uint32_t)(sb.ser.size() - at);
      x.sig_at = sb.sig.size();
      x.sig_len = (uint32_t)sig.size();
      sb.sig.append((const char*)sig.data(), sig.size());
      idr_of[(size_t)i] = iv;
      bool fresh = false;
      x.uid = slot.find_or_add(ip, (size_t)ni, (uint32_t)uniq.size(), fresh);
      if (fresh) uniq.push_back(iv);
    }
  }
  auto t_p3 = now();
  // (4) on the workers, per item: the fast / short flags, the batch-wide
  // identifier id, crypto_sign_open's split at byte 64 (message length);
  // offsets by a prefix sum over the kScanChunk chunks (chunk sums, a short
  // serial pass over them, then each chunk's offsets)
  std::string& fast = S.fast;
  std::string& shortv = S.shortv;
  std::vector<uint64_t>& off = S.off;
  std::vector<uint32_t>& uidx = S.uidx;
  fast.resize((size_t)n);
  shortv.resize((size_t)n);
  if (!staged) {  // (a staged batch's messages are placed already: its spans say where)
    off.resize((size_t)n + 1);
    off[0] = 0;
  }
  if (unique_form) uidx.resize((size_t)n);
  std::vector<uint64_t> csum((size_t)((n + kScanChunk - 1) / kScanChunk) + 1, 0);
  run_chunks(n, t, [&](int, Py_ssize_t a, Py_ssize_t b) {
    uint64_t sum = 0;
    for (Py_ssize_t i = a; i < b; ++i) {
      const ScanItem& x = it[(size_t)i];
      uint64_t len = 0;
      uint32_t u = 0xffffffffu;
      char f = 0, sh = 0;
      if (x.state == 1) {
        f = 1;
        u = x.buf < t ? to_global[x.buf][x.uid] : x.uid;  // bufs[t]: redone under the GIL, id already global
        const uint64_t ls = x.sig_len, lm = x.ser_len;
        if (ls + lm < 64)
          sh = 1;  // crypto_sign_open: smlen < 64 rejects
        else
          len = ls + lm - 64;
      }
      fast[(size_t)i] = f;
      shortv[(size_t)i] = sh;
      if (unique_form) uidx[(size_t)i] = u;
      if (!staged) off[(size_t)i + 1] = len;
      sum += len;
    }
    csum[(size_t)(a / kScanChunk) + 1] = sum;  // (one call over [0, n) when not chunked: csum[1])
  });
  if (!staged) {
    for (size_t c = 1; c < csum.size(); ++c) csum[c] += csum[c - 1];
    run_chunks(n, t, [&](int, Py_ssize_t a, Py_ssize_t b) {
      uint64_t at = csum[(size_t)(a / kScanChunk)];
      for (Py_ssize_t i = a; i < b; ++i) off[(size_t)i + 1] = at += off[(size_t)i + 1];
    });
  }
  // (5) sig64 and the messages, written by the workers into the result objects (a deferred
  // scan leaves this to pack_range, stretch by stretch, so the caller can queue each stretch's
  // DMA while the next one packs)
  char* dmsg = nullptr;
  if (staged) {  // the messages are in place; the spans say where
    Py_INCREF(out_msg);
    refs.o_msg = out_msg;
    PyObject* ul = PyList_New((Py_ssize_t)uniq.size());
    if (!ul) return nullptr;
    for (size_t u = 0; u < uniq.size(); ++u) {
      Py_INCREF(uniq[u]);
      PyList_SET_ITEM(ul, (Py_ssize_t)u, uniq[u]);
    }
    if (prof) {
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      fprintf(stderr,
              "scan (staged): n=%zd threads=%d  workers %.0f us, merge %.0f us (partitions %.0f, order %.0f, remap "
              "%.0f), bookkeeping %.0f us\n",
              n, t, us(t_start, t_p1), us(t_p1, t_p2), us(t_p1, t_m1), us(t_m1, t_m2), us(t_m2, t_p2),
              us(t_p3, now()));
    }
    // speculation: the key id used per distinct identifier (uint32 bytes), or None; parts_ok: every
    // part's kernels were queued
    PyObject* su = kmap ? PyBytes_FromStringAndSize((const char*)spec_u.data(), (Py_ssize_t)(spec_u.size() * 4))
                        : (Py_INCREF(Py_None), Py_None);
    if (!su) {
      Py_DECREF(ul);
      return nullptr;
    }
    PyObject* parts_ok = part_fn && !copier.part_failed && copier.next_part * part_items >= (uint64_t)n ? Py_True
                                                                                                      : Py_False;
    // staged_bytes: the message bytes the chunks reserved (the largest span end; sizes the next buffer)
    const unsigned long long staged_bytes = scursor.load() & ((1ull << kSeqShift) - 1);
    if (spans_p != S.spans.data())  // written in place: the caller's buffer is the result
      return Py_BuildValue("(y#y#NOOOy#ONOK)", fast.data(), (Py_ssize_t)n, (const char*)uidx.data(),
                           (Py_ssize_t)(uidx.size() * 4), ul, o_sig, out_msg, out_spans, shortv.data(), (Py_ssize_t)n,
                           staged_ok.load() ? Py_True : Py_False, su, parts_ok, staged_bytes);
    return Py_BuildValue("(y#y#NOOy#y#ONOK)", fast.data(), (Py_ssize_t)n, (const char*)uidx.data(),
                         (Py_ssize_t)(uidx.size() * 4), ul, o_sig, out_msg, (const char*)S.spans.data(),
                         (Py_ssize_t)(S.spans.size() * 8), shortv.data(), (Py_ssize_t)n,
                         staged_ok.load() ? Py_True : Py_False, su, parts_ok, staged_bytes);
  }
  PyObject* o_msg = refs.o_msg = out_buffer(out_msg, (Py_ssize_t)off[(size_t)n], &dmsg);
  PyObject* ret = nullptr;
  if (o_msg) {
    PackState P;
    P.S = &S;
    P.dsig = dsig;
    P.dmsg = dmsg;
    P.sig_slot = sig_slot;
    P.t = t;
    P.n = n;
    PyObject* handle = nullptr;
    if (defer) {
      PackState* hp = new PackState(P);
      handle = PyCapsule_New(hp, "edv.pack", pack_capsule_free);
      if (!handle) {
        delete hp;
        return nullptr;
      }
      hp->o_sig = o_sig;
      hp->o_msg = o_msg;
      Py_INCREF(o_sig);
      Py_INCREF(o_msg);
      held.s = nullptr;  // the handle owns the scratch now
    } else {
      pack_items(P, 0, n);
    }
    if (prof) {
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      fprintf(stderr,
              "scan: n=%zd threads=%d  workers %.0f us, merge %.0f us (partitions %.0f, order %.0f, remap %.0f), under "
              "the GIL %.0f us, pack %.0f us\n",
              n, t, us(t_start, t_p1), us(t_p1, t_p2), us(t_p1, t_m1), us(t_m1, t_m2), us(t_m2, t_p2), us(t_p2, t_p3),
              us(t_p3, now()));
    }
    if (unique_form) {
      PyObject* ul = PyList_New((Py_ssize_t)uniq.size());
      if (ul) {
        for (size_t u = 0; u < uniq.size(); ++u) {
          Py_INCREF(uniq[u]);
          PyList_SET_ITEM(ul, (Py_ssize_t)u, uniq[u]);
        }
        if (handle)
          ret = Py_BuildValue("(y#y#OOOy#y#N)", fast.data(), (Py_ssize_t)n, (const char*)uidx.data(),
                              (Py_ssize_t)(uidx.size() * 4), ul, o_sig, o_msg, (const char*)off.data(),
                              (Py_ssize_t)(off.size() * 8), shortv.data(), (Py_ssize_t)n, handle);
        else
          ret = Py_BuildValue("(y#y#OOOy#y#)", fast.data(), (Py_ssize_t)n, (const char*)uidx.data(),
                              (Py_ssize_t)(uidx.size() * 4), ul, o_sig, o_msg, (const char*)off.data(),
                              (Py_ssize_t)(off.size() * 8), shortv.data(), (Py_ssize_t)n);
        Py_DECREF(ul);
      } else {
        Py_XDECREF(handle);
      }
    } else {
      PyObject* idrs = PyList_New(n);
      if (idrs) {
        for (Py_ssize_t i = 0; i < n; ++i) {
          PyObject* idr = it[(size_t)i].state == 1 ? idr_of[(size_t)i] : Py_None;
          Py_INCREF(idr);
          PyList_SET_ITEM(idrs, i, idr);
        }
        ret = Py_BuildValue("(y#OOOy#y#)", fast.data(), (Py_ssize_t)n, idrs, o_sig, o_msg, (const char*)off.data(),
                            (Py_ssize_t)(off.size() * 8), shortv.data(), (Py_ssize_t)n);
        Py_DECREF(idrs);
      }
    }
  }
  return ret;
}

// No C++ exception reaches the interpreter: a worker's bad_alloc (buffers of a
// very large batch) becomes MemoryError once every worker has stopped
// (HostPool::run rethrows on the caller only after the helpers are done).
PyObject* scan_impl(PyObject* args, bool unique_form) {
  PyRefs refs;
  try {
    return scan_impl_body(args, unique_form, refs);
  } catch (const std::bad_alloc&) {
    return PyErr_NoMemory();
  } catch (const std::exception& e) {
    PyErr_Format(PyExc_RuntimeError, "scan_batch: %s", e.what());
    return nullptr;
  } catch (...) {
    PyErr_SetString(PyExc_RuntimeError, "scan_batch: native error");
    return nullptr;
  }
}

PyObject* py_scan_batch(PyObject*, PyObject* args) { return scan_impl(args, false); }
PyObject* py_scan_batch_u(PyObject*, PyObject* args) { return scan_impl(args, true); }

// Phase (5) for items [lo, hi): their messages at off[i] and the signature slots the workers did
// not write (raw signatures, zeroed slots of items that take the Python path or are short).
void pack_items(const PackState& P, Py_ssize_t lo, Py_ssize_t hi) {
  const ScanScratch& S = *P.S;
  const std::vector<ScanItem>& it = S.it;
  const std::vector<ScanBuf>& bufs = S.bufs;
  const std::vector<uint64_t>& off = S.off;
  const std::string& shortv = S.shortv;
  const int sig_slot = P.sig_slot;
  const bool slots = sig_slot == kSigSlot;
  char* dsig = P.dsig;
  char* dmsg = P.dmsg;
  run_chunks(hi - lo, P.t, [&](int, Py_ssize_t a0, Py_ssize_t b0) {
    for (Py_ssize_t i = lo + a0; i < lo + b0; ++i) {
      const ScanItem& x = it[(size_t)i];
      char* ds = dsig + (size_t)i * sig_slot;
      if (x.state == 1 && x.text) {  // slot written by the worker in (1)
        memcpy(dmsg + off[(size_t)i], bufs[x.buf].ser.data() + x.ser_at, x.ser_len);
        continue;
      }
      if (slots) memset(ds + 64, 0, (size_t)sig_slot - 64);  // slot[95] = 0: raw R || S in bytes 0..63
      if (x.state != 1 || shortv[(size_t)i]) {
        memset(ds, 0, 64);
        continue;
      }
      const ScanBuf& sb = bufs[x.buf];
      const char* sr = sb.ser.data() + x.ser_at;
      const size_t ls = x.sig_len, lm = x.ser_len;
      char* dm = dmsg + off[(size_t)i];
      const char* sg = sb.sig.data() + x.sig_at;
      if (ls >= 64) {  // sm[64:] = sig[64:] || ser
        memcpy(ds, sg, 64);
        memcpy(dm, sg + 64, ls - 64);
        memcpy(dm + (ls - 64), sr, lm);
      } else {
        memcpy(ds, sg, ls);
        memcpy(ds + ls, sr, 64 - ls);
        memcpy(dm, sr + (64 - ls), lm - (64 - ls));
      }
    }
  });
}

// pack_range(handle, lo, hi): phase (5) of a deferred scan_batch_u for items [lo, hi).
PyObject* py_pack_range(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_ssize_t lo, hi;
  if (!PyArg_ParseTuple(args, "Onn", &cap, &lo, &hi)) return nullptr;
  PackState* P = (PackState*)PyCapsule_GetPointer(cap, "edv.pack");
  if (!P) return nullptr;
  if (lo < 0 || hi > P->n || lo > hi) {
    PyErr_SetString(PyExc_ValueError, "pack_range: range outside the batch");
    return nullptr;
  }
  try {
    pack_items(*P, lo, hi);
  } catch (const std::bad_alloc&) {
    return PyErr_NoMemory();
  } catch (...) {
    PyErr_SetString(PyExc_RuntimeError, "pack_range: native error");
    return nullptr;
  }
  Py_RETURN_NONE;
}

// repack_spans(buf, spans) -> (msgs, off): a staged scan's messages (item i at buf[start[i]:end[i]],
// spans = starts[n] then ends[n], uint64) laid out contiguously with offsets, for the ordinary path.
PyObject* py_repack_spans(PyObject*, PyObject* args) {
  Py_buffer bb, bs;
  if (!PyArg_ParseTuple(args, "y*y*", &bb, &bs)) return nullptr;
  PyObject* ret = nullptr;
  const Py_ssize_t n = bs.len / 16;
  const uint64_t* st = (const uint64_t*)bs.buf;
  const uint64_t* en = st + n;
  std::vector<uint64_t> off((size_t)n + 1, 0);
  bool ok = bs.len % 16 == 0;
  for (Py_ssize_t i = 0; i < n && ok; ++i) {
    ok = st[i] <= en[i] && en[i] <= (uint64_t)bb.len;
    off[(size_t)i + 1] = off[(size_t)i] + (ok ? en[i] - st[i] : 0);
  }
  if (!ok) {
    PyErr_SetString(PyExc_ValueError, "repack_spans: span outside the buffer");
  } else {
    PyObject* m = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)off[(size_t)n]);
    if (m) {
      char* d = PyBytes_AS_STRING(m);
      for (Py_ssize_t i = 0; i < n; ++i) memcpy(d + off[(size_t)i], (const char*)bb.buf + st[i], en[i] - st[i]);
      ret = Py_BuildValue("(Ny#)", m, (const char*)off.data(), (Py_ssize_t)(off.size() * 8));
    }
  }
  PyBuffer_Release(&bb);
  PyBuffer_Release(&bs);
  return ret;
}

// results_from(codes, uidx, uniq) -> list: item i is uniq[uidx[i]] where
// codes[i] == 1 (verified: authenticate() returns the identifier), None
// elsewhere (the caller fills those in).
PyObject* py_results_from(PyObject*, PyObject* args) {
  Py_buffer bc, bu;
  PyObject* uniq;
  if (!PyArg_ParseTuple(args, "y*y*O", &bc, &bu, &uniq)) return nullptr;
  PyObject* ret = nullptr;
  const Py_ssize_t n = bc.len;
  if (!PyList_CheckExact(uniq) || bu.len != n * 4) {
    PyErr_SetString(PyExc_ValueError, "results_from: codes / uidx / uniq mismatch");
  } else {
    const uint8_t* c = (const uint8_t*)bc.buf;
    const uint32_t* u = (const uint32_t*)bu.buf;
    const Py_ssize_t nu = PyList_GET_SIZE(uniq);
    bool ok = true;
    for (Py_ssize_t i = 0; i < n && ok; ++i) ok = c[i] != 1 || (Py_ssize_t)u[i] < nu;
    if (!ok) {
      PyErr_SetString(PyExc_ValueError, "results_from: identifier index out of range");
    } else if ((ret = PyList_New(n))) {
      for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* o = c[i] == 1 ? PyList_GET_ITEM(uniq, u[i]) : Py_None;
        Py_INCREF(o);
        PyList_SET_ITEM(ret, i, o);
      }
    }
  }
  PyBuffer_Release(&bc);
  PyBuffer_Release(&bu);
  return ret;
}

// results_ok(ok, short, uidx, uniq) -> (results, failed): a steady-state batch's result list in
// one pass -- results[i] = uniq[uidx[i]] when ok[i] and not short[i], else None, with the
// indices of those failures (the caller puts InvalidSignature there).  ok / short: one byte
// per request (0 / nonzero).
// fails (optional): the objects to put at the failures instead of None, one per failure in index
// order (the caller's InvalidSignature instances, made BEFORE this list exists: allocating them
// after it would let the collector's young-generation passes walk the fresh list's items).
PyObject* py_results_ok(PyObject*, PyObject* args) {
  Py_buffer bo, bs, bu;
  PyObject* uniq;
  PyObject* fails = nullptr;
  if (!PyArg_ParseTuple(args, "y*y*y*O|O", &bo, &bs, &bu, &uniq, &fails)) return nullptr;
  struct Rel {
    Py_buffer *a, *b, *c;
    ~Rel() {
      PyBuffer_Release(a);
      PyBuffer_Release(b);
      PyBuffer_Release(c);
    }
  } rel{&bo, &bs, &bu};
  const Py_ssize_t n = bo.len;
  if (!PyList_CheckExact(uniq) || bs.len != n || bu.len != n * 4) {
    PyErr_SetString(PyExc_ValueError, "results_ok: ok / short / uidx / uniq mismatch");
    return nullptr;
  }
  const uint8_t* ok = (const uint8_t*)bo.buf;
  const uint8_t* sh = (const uint8_t*)bs.buf;
  const uint32_t* u = (const uint32_t*)bu.buf;
  const Py_ssize_t nu = PyList_GET_SIZE(uniq);
  PyObject** uitems = ((PyListObject*)uniq)->ob_item;
  PyObject* res = PyList_New(n);
  if (!res) return nullptr;
  // The list's items are written by the scan's worker threads (pointers only: no reference count
  // is touched off this thread); each worker counts the references it stored per identifier and
  // the failures it saw, and this thread adds the counts afterwards -- a 1M-request batch's result
  // list in a fraction of the serial pass.  (The list is not visible to any other Python code
  // until it is returned.)  Many distinct identifiers: the serial pass.
  const int t = nu <= (1 << 16) ? scan_threads(n, 0) : 1;
  std::vector<std::vector<uint32_t>> cnt((size_t)t);
  std::vector<std::vector<Py_ssize_t>> bad((size_t)t);
  std::atomic<bool> range_err{false};
  PyObject** items = ((PyListObject*)res)->ob_item;
  run_chunks(n, t, [&](int w, Py_ssize_t a, Py_ssize_t b) {
    std::vector<uint32_t>& c = cnt[(size_t)w];
    if (c.empty()) c.assign((size_t)nu + 1, 0);  // [nu] counts None
    std::vector<Py_ssize_t>& f = bad[(size_t)w];
    for (Py_ssize_t i = a; i < b; ++i) {
      const bool pass = ok[i] && !sh[i];
      if (pass && (Py_ssize_t)u[i] >= nu) {
        range_err = true;
        items[i] = Py_None;
        ++c[(size_t)nu];
        continue;
      }
      if (pass) {
        items[i] = uitems[u[i]];
        ++c[u[i]];
      } else {
        items[i] = Py_None;
        ++c[(size_t)nu];
        f.push_back(i);
      }
    }
  });
  // the workers' counts summed first (sequential arrays), then ONE reference update per identifier:
  // adding each worker's counts to the objects directly touched every identifier once per worker
  // (~30k cold objects x 16 workers in a churning batch)
  std::vector<uint64_t> tot((size_t)nu + 1, 0);
  for (const std::vector<uint32_t>& c : cnt) {
    if (c.empty()) continue;
    for (Py_ssize_t k = 0; k <= nu; ++k) tot[(size_t)k] += c[(size_t)k];
  }
  for (Py_ssize_t k = 0; k < nu; ++k)
    if (tot[(size_t)k]) Py_SET_REFCNT(uitems[k], Py_REFCNT(uitems[k]) + (Py_ssize_t)tot[(size_t)k]);
  Py_SET_REFCNT(Py_None, Py_REFCNT(Py_None) + (Py_ssize_t)tot[(size_t)nu]);
  if (range_err) {
    Py_DECREF(res);
    PyErr_SetString(PyExc_ValueError, "results_ok: identifier index out of range");
    return nullptr;
  }
  // failures in index order (the chunks of a worker ascend; the workers' lists are merged)
  std::vector<Py_ssize_t> all;
  for (const std::vector<Py_ssize_t>& f : bad) all.insert(all.end(), f.begin(), f.end());
  std::sort(all.begin(), all.end());
  if (fails && fails != Py_None && PyList_CheckExact(fails) && PyList_GET_SIZE(fails) == (Py_ssize_t)all.size()) {
    for (size_t j = 0; j < all.size(); ++j) {  // (items[i] holds Py_None: its reference moves to the count below)
      PyObject* o = PyList_GET_ITEM(fails, (Py_ssize_t)j);
      Py_INCREF(o);
      items[all[j]] = o;
    }
    Py_SET_REFCNT(Py_None, Py_REFCNT(Py_None) - (Py_ssize_t)all.size());
  }
  PyObject* failed = PyList_New((Py_ssize_t)all.size());
  if (!failed) {
    Py_DECREF(res);
    return nullptr;
  }
  for (size_t j = 0; j < all.size(); ++j) {
    PyObject* k = PyLong_FromSsize_t(all[j]);
    if (!k) {
      Py_DECREF(res);
      Py_DECREF(failed);
      return nullptr;
    }
    PyList_SET_ITEM(failed, (Py_ssize_t)j, k);
  }
  PyObject* ret = PyTuple_Pack(2, res, failed);
  Py_DECREF(res);
  Py_DECREF(failed);
  return ret;
}

// gather_u32(table, idx) -> bytearray: out[i] = table[idx[i]] (uint32 LE both), the key id of
// every request from its identifier's (one pass; numpy's fancy indexing widens the index
// array to intp first).  ValueError on an index past the table.
PyObject* py_gather_u32(PyObject*, PyObject* args) {
  Py_buffer bt, bi;
  PyObject* out = Py_None;
  if (!PyArg_ParseTuple(args, "y*y*|O", &bt, &bi, &out)) return nullptr;
  struct Rel {
    Py_buffer *a, *b;
    ~Rel() {
      PyBuffer_Release(a);
      PyBuffer_Release(b);
    }
  } rel{&bt, &bi};
  const Py_ssize_t nt = bt.len / 4, n = bi.len / 4;
  if (bt.len % 4 || bi.len % 4) {
    PyErr_SetString(PyExc_ValueError, "gather_u32: buffers of uint32 expected");
    return nullptr;
  }
  // out: a bytearray reused from call to call (grown, never shrunk: a fresh 4 MB result per 1M
  // requests costs its page faults every batch); else a new bytearray of exactly n ids
  char* data = nullptr;
  PyObject* ret = out != Py_None ? out_buffer(out, n * 4, &data) : PyByteArray_FromStringAndSize(nullptr, n * 4);
  if (!ret) return nullptr;
  if (!data) data = PyByteArray_Check(ret) ? PyByteArray_AS_STRING(ret) : PyBytes_AS_STRING(ret);
  const uint32_t* t = (const uint32_t*)bt.buf;
  const uint32_t* ix = (const uint32_t*)bi.buf;
  uint32_t* o = (uint32_t*)data;
  std::atomic<uint32_t> bad{0};
  run_chunks(n, n >= (1 << 18) ? scan_threads(n / 8, 0) : 1, [&](int, Py_ssize_t a, Py_ssize_t b) {
    uint32_t bd = 0;
    for (Py_ssize_t i = a; i < b; ++i) {
      const uint32_t k = ix[i];
      bd |= (uint32_t)(k >= (uint32_t)nt);
      o[i] = k < (uint32_t)nt ? t[k] : 0u;
    }
    if (bd) bad = 1;
  }, 1 << 16);
  if (bad) {
    Py_DECREF(ret);
    PyErr_SetString(PyExc_ValueError, "gather_u32: index out of range");
    return nullptr;
  }
  return ret;
}

// gather_items(sig, msgbuf, off, idx, stride=64) -> (sig', msgbuf', off'): the
// items idx (uint32 LE) of a split batch, repacked contiguously; stride is the
// signature record size (64 = R || S, 96 = edverify.h signature slots).
// gather_spans(sig, msgbuf, spans, idx_u32, stride=96) -> (sig_k, msg_k, off_k): gather_items over a
// staged batch, whose item i's message is msgbuf[starts[i], ends[i]) (spans = starts[n] then ends[n],
// uint64): the items of a staged batch that take another path.
PyObject* py_gather_spans(PyObject*, PyObject* args) {
  Py_buffer bs, bm, bp, bi;
  Py_ssize_t stride = 64;
  if (!PyArg_ParseTuple(args, "y*y*y*y*|n", &bs, &bm, &bp, &bi, &stride)) return nullptr;
  const uint64_t* st = (const uint64_t*)bp.buf;
  const uint32_t* idx = (const uint32_t*)bi.buf;
  const Py_ssize_t n = bp.len / 16, k = bi.len / 4;
  const uint64_t* en = st + n;
  bool ok = (stride == 64 || stride == kSigSlot) && bp.len % 16 == 0 && bs.len >= n * stride;
  std::string sig, msg;
  std::vector<uint64_t> o((size_t)k + 1, 0);
  if (ok) sig.assign((size_t)k * (size_t)stride, '\0');
  for (Py_ssize_t j = 0; j < k && ok; ++j) {
    const uint32_t i = idx[j];
    if ((Py_ssize_t)i >= n || en[i] < st[i] || en[i] > (uint64_t)bm.len) {
      ok = false;
      break;
    }
    memcpy(&sig[(size_t)j * stride], (const char*)bs.buf + (size_t)i * stride, (size_t)stride);
    msg.append((const char*)bm.buf + st[i], en[i] - st[i]);
    o[(size_t)j + 1] = msg.size();
  }
  PyBuffer_Release(&bs);
  PyBuffer_Release(&bm);
  PyBuffer_Release(&bp);
  PyBuffer_Release(&bi);
  if (!ok) {
    PyErr_SetString(PyExc_ValueError, "gather_spans: stride, index or spans out of range");
    return nullptr;
  }
  return Py_BuildValue("(y#y#y#)", sig.data(), (Py_ssize_t)sig.size(), msg.data(), (Py_ssize_t)msg.size(),
                       (const char*)o.data(), (Py_ssize_t)(o.size() * 8));
}

// keys_known(clients, fast_keys, identifiers, field) -> (keys, holes): the authenticator's
// per-identifier key resolution (SimpleAuthNr.getVerkey, client_authn.py:142-154, then the
// remembered DidVerifier key) for the identifiers whose answer needs no Python: clients[idr] an
// exact non-empty dict, its `field` entry the very verkey object fast_keys[idr] = (verkey, key)
// remembers.  keys[j] = that key bytes, else None; holes = the j of the Nones (the caller's Python
// path: getVerkey's state lookup, its exceptions, a changed verkey).  Only for an exact-dict
// `clients` read by the known getVerkey (the caller checks); nothing here has side effects.
PyObject* py_keys_known(PyObject*, PyObject* args) {
  PyObject *clients, *fk, *idrs, *field;
  if (!PyArg_ParseTuple(args, "O!O!O!O", &PyDict_Type, &clients, &PyDict_Type, &fk, &PyList_Type, &idrs, &field))
    return nullptr;
  if (!PyDict_CheckExact(clients) || !PyDict_CheckExact(fk) || !PyList_CheckExact(idrs)) {
    PyErr_SetString(PyExc_TypeError, "keys_known: exact dicts and a list");
    return nullptr;
  }
  const Py_ssize_t n = PyList_GET_SIZE(idrs);
  PyObject* keys = PyList_New(n);
  PyObject* holes = keys ? PyList_New(0) : nullptr;
  if (!holes) {
    Py_XDECREF(keys);
    return nullptr;
  }
#ifdef EDV_HAVE_DK
  // A churning batch brings ~30k identifiers whose clients / fast_keys entries (100k-entry dicts)
  // and nym dicts are cold: each lookup below is a chain of dependent cache misses.  The
  // identifiers D, 2D, 3D ahead walk the same chains one link per iteration (hash -> index slot ->
  // entry -> key, value and the nym dict's keys), with prefetches only, so the lookups find them
  // cached.  Reads stay in bounds (slot < size, entry < nentries); a stale guess only wastes a
  // prefetch.
  constexpr Py_ssize_t kD = 8;
  static const bool prefetch = !(getenv("EDV_KEYS_PREFETCH") && getenv("EDV_KEYS_PREFETCH")[0] == '0');  // A/B
  const auto slot_of = [](PyObject* d, Py_hash_t h, const DkEntry*& ent, Py_ssize_t& ne) -> Py_ssize_t {
    const DkHead* k = (const DkHead*)((const PyDictObject*)d)->ma_keys;
    ent = dk_entries(d, ne);
    if (!ent) return -1;
    const Py_ssize_t sz = k->size, s = (Py_ssize_t)((size_t)h & (size_t)(sz - 1));
    const Py_ssize_t ix = sz <= 0xff ? ((const int8_t*)k->idx)[s]
                          : sz <= 0xffff ? ((const int16_t*)k->idx)[s]
                          : sz <= 0xffffffffLL ? ((const int32_t*)k->idx)[s] : ((const int64_t*)k->idx)[s];
    return ix >= 0 && ix < ne ? ix : -1;
  };
  const auto pf_slot = [](PyObject* d, Py_hash_t h) {
    if (((const PyDictObject*)d)->ma_values) return;
    const DkHead* k = (const DkHead*)((const PyDictObject*)d)->ma_keys;
    const Py_ssize_t sz = k->size, w = sz <= 0xff ? 1 : sz <= 0xffff ? 2 : sz <= 0xffffffffLL ? 4 : 8;
    __builtin_prefetch(k->idx + ((size_t)h & (size_t)(sz - 1)) * w);
  };
  const auto hash_of = [](PyObject* s) -> Py_hash_t {  // cached after the first call; -1: not an exact str
    if (!PyUnicode_CheckExact(s)) return -1;
    Py_hash_t h = ((PyASCIIObject*)s)->hash;
    if (h == -1) {
      h = PyObject_Hash(s);
      if (h == -1) PyErr_Clear();
    }
    return h;
  };
#endif
  for (Py_ssize_t j = 0; j < n; ++j) {
    PyObject* idr = PyList_GET_ITEM(idrs, j);
    PyObject* key = nullptr;
#ifdef EDV_HAVE_DK
    const auto hash_at = [&](Py_ssize_t i) -> Py_hash_t {
      PyObject* s = PyList_GET_ITEM(idrs, i);
      return PyUnicode_CheckExact(s) ? ((PyASCIIObject*)s)->hash : -1;
    };
    const DkEntry* ent;
    Py_ssize_t ne, ix;
    if (prefetch && j + 4 * kD < n) {  // link 1: the index slots
      const Py_hash_t h = hash_of(PyList_GET_ITEM(idrs, j + 4 * kD));
      if (h != -1) {
        pf_slot(clients, h);
        pf_slot(fk, h);
      }
    }
    if (prefetch && j + 3 * kD < n) {  // link 2: the entries
      const Py_hash_t h = hash_at(j + 3 * kD);
      if (h != -1) {
        if ((ix = slot_of(clients, h, ent, ne)) >= 0) __builtin_prefetch(&ent[ix]);
        if ((ix = slot_of(fk, h, ent, ne)) >= 0) __builtin_prefetch(&ent[ix]);
      }
    }
    if (prefetch && j + 2 * kD < n) {  // link 3: the keys, the nym dicts and the (verkey, key) tuples
      const Py_hash_t h = hash_at(j + 2 * kD);
      if (h != -1) {
        if ((ix = slot_of(clients, h, ent, ne)) >= 0 && ent[ix].h == h) {
          __builtin_prefetch(ent[ix].k);
          __builtin_prefetch(ent[ix].v);
        }
        if ((ix = slot_of(fk, h, ent, ne)) >= 0 && ent[ix].h == h) __builtin_prefetch(ent[ix].v);
      }
    }
    if (prefetch && j + kD < n) {  // link 4: the nym dicts' key tables and the tuples' key bytes
      const Py_hash_t h = hash_at(j + kD);
      if (h != -1) {
        if ((ix = slot_of(clients, h, ent, ne)) >= 0 && ent[ix].h == h && ent[ix].v &&
            Py_TYPE(ent[ix].v) == &PyDict_Type)
          __builtin_prefetch(((const PyDictObject*)ent[ix].v)->ma_keys);
        if ((ix = slot_of(fk, h, ent, ne)) >= 0 && ent[ix].h == h && ent[ix].v && PyTuple_CheckExact(ent[ix].v) &&
            PyTuple_GET_SIZE(ent[ix].v) == 2)
          __builtin_prefetch(PyTuple_GET_ITEM(ent[ix].v, 1));
      }
    }
#endif
    if (PyUnicode_CheckExact(idr)) {
      PyObject* nym = PyDict_GetItemWithError(clients, idr);  // borrowed
      if (nym && PyDict_CheckExact(nym) && PyDict_GET_SIZE(nym) > 0) {
        PyObject* vk = PyDict_GetItemWithError(nym, field);
        PyObject* e = vk ? PyDict_GetItemWithError(fk, idr) : nullptr;
        if (e && PyTuple_CheckExact(e) && PyTuple_GET_SIZE(e) == 2 && PyTuple_GET_ITEM(e, 0) == vk &&
            PyBytes_CheckExact(PyTuple_GET_ITEM(e, 1)))
          key = PyTuple_GET_ITEM(e, 1);
      }
      if (PyErr_Occurred()) {
        Py_DECREF(keys);
        Py_DECREF(holes);
        return nullptr;
      }
    }
    if (key) {
      Py_INCREF(key);
      PyList_SET_ITEM(keys, j, key);
    } else {
      Py_INCREF(Py_None);
      PyList_SET_ITEM(keys, j, Py_None);
      PyObject* jj = PyLong_FromSsize_t(j);
      if (!jj || PyList_Append(holes, jj) != 0) {
        Py_XDECREF(jj);
        Py_DECREF(keys);
        Py_DECREF(holes);
        return nullptr;
      }
      Py_DECREF(jj);
    }
  }
  return Py_BuildValue("(NN)", keys, holes);
}

#ifdef EDV_HAVE_DK
// A worker's dict lookup by an exact-str key, on CPython 3.10's combined table and probe
// sequence (Objects/dictobject.c lookdict): pure reads, no Python code, no reference counts.
// 1 found (*v borrowed), 0 absent, -1 not decidable here (a split table, a non-str or deleted key
// on the probe path with the same hash, a probe past the table) -- the caller's Python path then.
// The key's hash is computed here when not yet cached (a pure function of the text; the object
// is this worker's alone while the GIL holder waits in the same call).
int w_dict_get_str(PyObject* d, PyObject* key, PyObject** v) {
  if (Py_TYPE(d) != &PyDict_Type || !PyUnicode_CheckExact(key)) return -1;
  const PyDictObject* od = (const PyDictObject*)d;
  if (od->ma_values) return -1;
  Py_hash_t h = ((PyASCIIObject*)key)->hash;
  if (h == -1) {
    h = PyObject_Hash(key);  // unicode_hash: _Py_HashBytes over the data, cached in the object
    if (h == -1) return -1;
  }
  Py_ssize_t ne = 0;
  const DkEntry* ent = dk_entries(d, ne);
  if (!ent) return -1;
  const DkHead* k = (const DkHead*)od->ma_keys;
  const Py_ssize_t sz = k->size;
  const size_t mask = (size_t)sz - 1;
  size_t i = (size_t)h & mask, perturb = (size_t)h;
  for (Py_ssize_t probes = 0; probes <= sz; ++probes) {
    const Py_ssize_t ix = sz <= 0xff ? ((const int8_t*)k->idx)[i]
                          : sz <= 0xffff ? ((const int16_t*)k->idx)[i]
                          : sz <= 0xffffffffLL ? ((const int32_t*)k->idx)[i] : ((const int64_t*)k->idx)[i];
    if (ix == -1) return 0;  // DKIX_EMPTY
    if (ix >= 0) {
      if (ix >= ne) return -1;
      const DkEntry& e = ent[ix];
      if (e.k == key) {
        *v = e.v;
        return e.v ? 1 : 0;
      }
      if (e.h == h) {
        if (!e.k || !PyUnicode_CheckExact(e.k)) return -1;
        if (w_str_eq(e.k, key)) {
          *v = e.v;
          return e.v ? 1 : 0;
        }
      }
    }
    perturb >>= 5;  // PERTURB_SHIFT
    i = (i * 5 + perturb + 1) & mask;
  }
  return -1;
}
#endif

#ifdef EDV_HAVE_DK
// keys_known_flat's prefetch pipeline for identifier j of a worker's range [.., b): the link of
// the identifiers 4d, 3d, 2d and d ahead (index slots; entries; the entries' key texts and values;
// the nym dicts' tables and the tuples' key bytes).  Only the hash computation writes (into the
// identifier's own cached hash, as the lookup would: the worker's own item).
inline void keys_prefetch_links(PyObject* clients, PyObject* fk, PyObject** items, Py_ssize_t j, Py_ssize_t b,
                                Py_ssize_t d) {
  const auto idx_of = [](PyObject* dct, Py_hash_t h, const DkEntry*& ent) -> Py_ssize_t {
    if (((const PyDictObject*)dct)->ma_values) return -1;
    Py_ssize_t ne = 0;
    ent = dk_entries(dct, ne);
    if (!ent) return -1;
    const DkHead* k = (const DkHead*)((const PyDictObject*)dct)->ma_keys;
    const Py_ssize_t sz = k->size, s = (Py_ssize_t)((size_t)h & (size_t)(sz - 1));
    const Py_ssize_t ix = sz <= 0xff ? ((const int8_t*)k->idx)[s]
                          : sz <= 0xffff ? ((const int16_t*)k->idx)[s]
                          : sz <= 0xffffffffLL ? ((const int32_t*)k->idx)[s] : ((const int64_t*)k->idx)[s];
    return ix >= 0 && ix < ne ? ix : -1;
  };
  const auto cached_hash = [&](Py_ssize_t i) -> Py_hash_t {
    PyObject* s = items[i];
    return PyUnicode_CheckExact(s) ? ((PyASCIIObject*)s)->hash : -1;
  };
  const DkEntry* ent;
  Py_ssize_t ix;
  if (j + 4 * d < b) {  // link 1: the index slots (the hash computed now when not cached)
    PyObject* s = items[j + 4 * d];
    if (PyUnicode_CheckExact(s)) {
      Py_hash_t h = ((PyASCIIObject*)s)->hash;
      if (h == -1) h = PyObject_Hash(s);
      for (PyObject* dct : {clients, fk}) {
        if (h == -1 || ((const PyDictObject*)dct)->ma_values) continue;
        const DkHead* k = (const DkHead*)((const PyDictObject*)dct)->ma_keys;
        const Py_ssize_t sz = k->size, w = sz <= 0xff ? 1 : sz <= 0xffff ? 2 : sz <= 0xffffffffLL ? 4 : 8;
        __builtin_prefetch(k->idx + ((size_t)h & (size_t)(sz - 1)) * w);
      }
    }
  }
  if (j + 3 * d < b) {  // link 2: the entries
    const Py_hash_t h = cached_hash(j + 3 * d);
    if (h != -1)
      for (PyObject* dct : {clients, fk})
        if ((ix = idx_of(dct, h, ent)) >= 0) __builtin_prefetch(&ent[ix]);
  }
  if (j + 2 * d < b) {  // link 3: the entries' key texts (compared) and values (nym dict, tuple)
    const Py_hash_t h = cached_hash(j + 2 * d);
    if (h != -1)
      for (PyObject* dct : {clients, fk})
        if ((ix = idx_of(dct, h, ent)) >= 0 && ent[ix].h == h) {
          if (ent[ix].k != items[j + 2 * d]) __builtin_prefetch(ent[ix].k);
          __builtin_prefetch(ent[ix].v);
        }
  }
  if (j + d < b) {  // link 4: the nym dict's table, the tuple's key bytes
    const Py_hash_t h = cached_hash(j + d);
    if (h != -1) {
      if ((ix = idx_of(clients, h, ent)) >= 0 && ent[ix].h == h && ent[ix].v && Py_TYPE(ent[ix].v) == &PyDict_Type)
        __builtin_prefetch(((const PyDictObject*)ent[ix].v)->ma_keys);
      if ((ix = idx_of(fk, h, ent)) >= 0 && ent[ix].h == h && ent[ix].v && PyTuple_CheckExact(ent[ix].v) &&
          PyTuple_GET_SIZE(ent[ix].v) == 2)
        __builtin_prefetch(PyTuple_GET_ITEM(ent[ix].v, 1));
    }
  }
}
#endif

// keys_known_flat(clients, fast_keys, identifiers, field) -> (keys, holes, flat): keys_known on the
// scan's worker pool, plus the keys' bytes in one buffer (flat[32 j .. 32 j + 32) = keys[j]; zeros
// at the holes, which include any key that is not 32 bytes) so the key store lookup and the general path's key array need no
// pass over the key objects.  A churning batch's ~30k identifiers are chains of cache misses in
// 100k-entry dicts: ~7.5 ms on one thread (keys_known, prefetched), a fraction of it on the pool.
// Each worker takes the references it hands out with atomic increments (only this call's workers
// touch reference counts while it runs).  Identifiers a worker cannot decide without the
// interpreter are holes, as in keys_known.  Outside CPython 3.10's layout: keys_known's serial
// pass, then the flat copy.
PyObject* py_keys_known_flat(PyObject* self, PyObject* args) {
  PyObject *clients, *fk, *idrs, *field;
  if (!PyArg_ParseTuple(args, "O!O!O!O", &PyDict_Type, &clients, &PyDict_Type, &fk, &PyList_Type, &idrs, &field))
    return nullptr;
  if (!PyDict_CheckExact(clients) || !PyDict_CheckExact(fk) || !PyList_CheckExact(idrs)) {
    PyErr_SetString(PyExc_TypeError, "keys_known_flat: exact dicts and a list");
    return nullptr;
  }
  const Py_ssize_t n = PyList_GET_SIZE(idrs);
  PyObject* flat = PyBytes_FromStringAndSize(nullptr, 32 * n);
  if (!flat) return nullptr;
  char* fp = PyBytes_AS_STRING(flat);
#ifdef EDV_HAVE_DK
  if (PyUnicode_CheckExact(field) && ((PyASCIIObject*)field)->hash != -1 && n >= 1024) {
    std::vector<PyObject*> got((size_t)n, nullptr);
    std::vector<uint8_t> undecided((size_t)n, 0);
    PyObject** items = ((PyListObject*)idrs)->ob_item;
    static const bool prefetch = !(getenv("EDV_KEYS_PREFETCH") && getenv("EDV_KEYS_PREFETCH")[0] == '0');  // A/B
    run_chunks(n, scan_threads(n, 0), [&](int, Py_ssize_t a, Py_ssize_t b) {
      // each lookup is a chain of ~10 dependent cache misses (index slot, entry, key text, nym
      // dict, its table, tuple, key bytes): the identifiers 1-4 x kPD ahead walk the same chains
      // one link per iteration with prefetches only (reads in bounds; a stale guess wastes a
      // prefetch), so the lookups below find their lines cached -- keys_known's pipeline, per worker
      constexpr Py_ssize_t kPD = 6;
      for (Py_ssize_t j = a; j < b; ++j) {
        if (prefetch) keys_prefetch_links(clients, fk, items, j, b, kPD);
        PyObject* idr = items[j];
        PyObject *nym = nullptr, *vk = nullptr, *e = nullptr, *key = nullptr;
        int r = w_dict_get_str(clients, idr, &nym);
        if (r == 1 && nym && PyDict_CheckExact(nym) && PyDict_GET_SIZE(nym) > 0) {
          r = w_dict_get_str(nym, field, &vk);
          if (r == 1 && vk) {
            r = w_dict_get_str(fk, idr, &e);
            if (r == 1 && e && PyTuple_CheckExact(e) && PyTuple_GET_SIZE(e) == 2 && PyTuple_GET_ITEM(e, 0) == vk &&
                PyBytes_CheckExact(PyTuple_GET_ITEM(e, 1)))
              key = PyTuple_GET_ITEM(e, 1);
          }
        }
        if (key && PyBytes_GET_SIZE(key) != 32) key = nullptr;  // (the Python path: rare)
        char* dst = fp + 32 * j;
        if (key) {
          __atomic_fetch_add(&key->ob_refcnt, 1, __ATOMIC_RELAXED);
          got[(size_t)j] = key;
          memcpy(dst, PyBytes_AS_STRING(key), 32);
        } else {
          memset(dst, 0, 32);
          undecided[(size_t)j] = 1;
        }
      }
    });
    PyObject* keys = PyList_New(n);
    PyObject* holes = keys ? PyList_New(0) : nullptr;
    bool ok = holes != nullptr;
    for (Py_ssize_t j = 0; j < n; ++j) {
      PyObject* key = got[(size_t)j];
      if (!keys) {
        Py_XDECREF(key);
        continue;
      }
      if (key) {
        PyList_SET_ITEM(keys, j, key);  // (the reference the worker took)
        continue;
      }
      Py_INCREF(Py_None);
      PyList_SET_ITEM(keys, j, Py_None);
      if (ok) {
        PyObject* jj = PyLong_FromSsize_t(j);
        ok = jj && PyList_Append(holes, jj) == 0;
        Py_XDECREF(jj);
      }
    }
    if (!ok) {
      Py_XDECREF(keys);
      Py_XDECREF(holes);
      Py_DECREF(flat);
      return nullptr;
    }
    return Py_BuildValue("(NNN)", keys, holes, flat);
  }
#endif
  PyObject* kh = py_keys_known(self, args);
  if (!kh) {
    Py_DECREF(flat);
    return nullptr;
  }
  PyObject* keys = PyTuple_GET_ITEM(kh, 0);
  for (Py_ssize_t j = 0; j < n; ++j) {
    PyObject* key = PyList_GET_ITEM(keys, j);
    if (PyBytes_CheckExact(key) && PyBytes_GET_SIZE(key) == 32)
      memcpy(fp + 32 * j, PyBytes_AS_STRING(key), 32);
    else
      memset(fp + 32 * j, 0, 32);
  }
  PyObject* out = Py_BuildValue("(OON)", keys, PyTuple_GET_ITEM(kh, 1), flat);
  Py_DECREF(kh);
  return out;
}

// A native index of 32-byte keys -> int64 (the key store's key -> slot id, mirrored by KeyStore so a
// batch's ~30k distinct keys are looked up in one call over the flat key buffer): open addressing,
// linear probing, tombstones, grown at 60 % use.
struct KeyIndex {
  struct E {
    uint64_t w[4];
    int64_t v;
    uint8_t st;  // 0 empty, 1 full, 2 deleted
  };
  std::vector<E> e = std::vector<E>(1024);
  size_t n = 0, used = 0;
  static uint64_t hash(const uint64_t* w) {  // keys are curve points: well mixed already
    uint64_t h = w[0] * 0x9E3779B97F4A7C15ull ^ w[1] ^ (w[2] * 0xC2B2AE3D27D4EB4Full) ^ w[3];
    return h ^ (h >> 29);
  }
  static bool eq(const E& x, const uint64_t* w) {
    return x.w[0] == w[0] && x.w[1] == w[1] && x.w[2] == w[2] && x.w[3] == w[3];
  }
  int64_t get(const uint64_t* w) const {
    const size_t mask = e.size() - 1;
    for (size_t s = hash(w) & mask;; s = (s + 1) & mask) {
      const E& x = e[s];
      if (x.st == 0) return -1;
      if (x.st == 1 && eq(x, w)) return x.v;
    }
  }
  void grow() {
    std::vector<E> old;
    old.swap(e);
    e.assign(old.size() * (2 * (n + 1) > old.size() / 2 ? 2 : 1), E{});
    used = n = 0;
    for (const E& x : old)
      if (x.st == 1) set(x.w, x.v);
  }
  void set(const uint64_t* w, int64_t v) {
    if (10 * (used + 1) > 6 * e.size()) grow();
    const size_t mask = e.size() - 1;
    size_t tomb = SIZE_MAX;
    for (size_t s = hash(w) & mask;; s = (s + 1) & mask) {
      E& x = e[s];
      if (x.st == 0) {
        E& y = tomb != SIZE_MAX ? e[tomb] : x;
        if (tomb == SIZE_MAX) ++used;
        memcpy(y.w, w, 32);
        y.v = v;
        y.st = 1;
        ++n;
        return;
      }
      if (x.st == 2 && tomb == SIZE_MAX) tomb = s;
      if (x.st == 1 && eq(x, w)) {
        x.v = v;
        return;
      }
    }
  }
  void del(const uint64_t* w) {
    const size_t mask = e.size() - 1;
    for (size_t s = hash(w) & mask;; s = (s + 1) & mask) {
      E& x = e[s];
      if (x.st == 0) return;
      if (x.st == 1 && eq(x, w)) {
        x.st = 2;
        --n;
        return;
      }
    }
  }
};
void key_index_free(PyObject* cap) { delete (KeyIndex*)PyCapsule_GetPointer(cap, "edv.keyindex"); }
KeyIndex* key_index_of(PyObject* cap) { return (KeyIndex*)PyCapsule_GetPointer(cap, "edv.keyindex"); }

PyObject* py_key_index(PyObject*, PyObject*) { return PyCapsule_New(new KeyIndex, "edv.keyindex", key_index_free); }

// key_index_set(index, keys, ids): keys 32 m bytes, ids m int64 (little-endian)
PyObject* py_key_index_set(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_buffer bk, bv;
  if (!PyArg_ParseTuple(args, "Oy*y*", &cap, &bk, &bv)) return nullptr;
  KeyIndex* ki = key_index_of(cap);
  const Py_ssize_t m = bk.len / 32;
  PyObject* ret = nullptr;
  if (ki && bk.len == 32 * m && bv.len == 8 * m) {
    for (Py_ssize_t j = 0; j < m; ++j) {
      uint64_t w[4];
      int64_t v;
      memcpy(w, (const char*)bk.buf + 32 * j, 32);
      memcpy(&v, (const char*)bv.buf + 8 * j, 8);
      ki->set(w, v);
    }
    ret = Py_None;
    Py_INCREF(ret);
  } else if (ki) {
    PyErr_SetString(PyExc_ValueError, "key_index_set: 32-byte keys and one int64 id each");
  }
  PyBuffer_Release(&bk);
  PyBuffer_Release(&bv);
  return ret;
}

PyObject* py_key_index_del(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_buffer bk;
  if (!PyArg_ParseTuple(args, "Oy*", &cap, &bk)) return nullptr;
  KeyIndex* ki = key_index_of(cap);
  PyObject* ret = nullptr;
  if (ki && bk.len % 32 == 0) {
    for (Py_ssize_t j = 0; j < bk.len / 32; ++j) {
      uint64_t w[4];
      memcpy(w, (const char*)bk.buf + 32 * j, 32);
      ki->del(w);
    }
    ret = Py_None;
    Py_INCREF(ret);
  } else if (ki) {
    PyErr_SetString(PyExc_ValueError, "key_index_del: 32-byte keys");
  }
  PyBuffer_Release(&bk);
  return ret;
}

PyObject* py_key_index_clear(PyObject*, PyObject* cap) {
  KeyIndex* ki = key_index_of(cap);
  if (!ki) return nullptr;
  *ki = KeyIndex();
  Py_RETURN_NONE;
}

PyObject* py_key_index_len(PyObject*, PyObject* cap) {
  KeyIndex* ki = key_index_of(cap);
  if (!ki) return nullptr;
  return PyLong_FromSize_t(ki->n);
}

// key_index_get(index, flat) -> bytes of m int64: the id of each 32-byte key of flat, -1 if absent
PyObject* py_key_index_get(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_buffer bk;
  if (!PyArg_ParseTuple(args, "Oy*", &cap, &bk)) return nullptr;
  KeyIndex* ki = key_index_of(cap);
  PyObject* out = nullptr;
  if (ki && bk.len % 32 == 0) {
    const Py_ssize_t m = bk.len / 32;
    out = PyBytes_FromStringAndSize(nullptr, 8 * m);
    if (out) {
      int64_t* o = (int64_t*)PyBytes_AS_STRING(out);
      const char* kb = (const char*)bk.buf;
      const KeyIndex& kx = *ki;
      // read-only probes: a churning batch's ~30k keys on the worker pool, each probe's slot
      // prefetched 8 keys ahead (the table is ~1.5 MB for 16k keys: a miss per key otherwise)
      run_chunks(m, m >= 8192 ? scan_threads(m, 0) : 1, [&](int, Py_ssize_t a, Py_ssize_t b) {
        const size_t mask = kx.e.size() - 1;
        for (Py_ssize_t j = a; j < b; ++j) {
          uint64_t w[4];
          if (j + 8 < b) {
            memcpy(w, kb + 32 * (j + 8), 32);
            __builtin_prefetch(&kx.e[KeyIndex::hash(w) & mask]);
          }
          memcpy(w, kb + 32 * j, 32);
          o[j] = kx.get(w);
        }
      });
    }
  } else if (ki) {
    PyErr_SetString(PyExc_ValueError, "key_index_get: 32-byte keys");
  }
  PyBuffer_Release(&bk);
  return out;
}

// The promotion policy's decayed verified-use counts (keystore.UseCounts) for 32-byte keys: key ->
// row (a KeyIndex) and per row the count, the epoch it was last counted at and the add() call that
// last counted it.  Rows are dense (a freed row is filled from the end).  A churning batch counts
// ~4k keys: the Python form spent ~2 ms on their dict probes and lists; here one pass over the
// batch's flat key buffer.
struct UseTable {
  KeyIndex idx;
  std::vector<std::array<uint64_t, 4>> key;
  std::vector<int64_t> u, e, t;
  std::vector<uint64_t> mark;  // scratch per row: the call that touched it, its sum, first position
  std::vector<int64_t> acc;
  std::vector<Py_ssize_t> first;
  int64_t tick = 0;
  uint64_t calls = 0;
  size_t cap;
  explicit UseTable(size_t c) : cap(c) {}
  size_t size() const { return u.size(); }
  // rows `gone` (distinct) are freed: the live rows past the new end move into the holes, both
  // in ascending order (the array form's _compact: the two forms keep the same row layout)
  void remove(std::vector<int64_t>& gone) {
    std::sort(gone.begin(), gone.end());
    for (int64_t r : gone) idx.del(key[(size_t)r].data());
    size_t n = size();
    std::vector<char> dead(n, 0);
    for (int64_t r : gone) dead[(size_t)r] = 1;
    size_t m = n - gone.size();
    size_t src = m;
    for (int64_t r : gone) {
      if ((size_t)r >= m) break;
      while (dead[src]) ++src;  // the next live row past the new end
      key[(size_t)r] = key[src];
      u[(size_t)r] = u[src];
      e[(size_t)r] = e[src];
      t[(size_t)r] = t[src];
      idx.set(key[(size_t)r].data(), r);
      ++src;
    }
    key.resize(m);
    u.resize(m);
    e.resize(m);
    t.resize(m);
  }
  // counts[j] verified uses of key j (counts below `floor` are not counted); returns the positions
  // j whose count reached hot_at, in input order (a key given twice: summed, reported once)
  std::vector<Py_ssize_t> add(const char* flat, const int64_t* counts, Py_ssize_t m, int64_t floor, int64_t now,
                              int64_t hot_at) {
    ++calls;
    std::vector<int64_t> rows((size_t)m, -1);
    for (Py_ssize_t j = 0; j < m; ++j) {
      const int64_t c = counts[j];
      if (c <= 0 || c < floor) continue;
      uint64_t w[4];
      memcpy(w, flat + 32 * j, 32);
      int64_t r = idx.get(w);
      if (r < 0) {
        r = (int64_t)size();
        idx.set(w, r);
        key.push_back({w[0], w[1], w[2], w[3]});
        u.push_back(0);
        e.push_back(now);
        t.push_back(0);
      }
      if (mark.size() <= (size_t)r) {
        mark.resize(size() * 2, 0);
        acc.resize(mark.size());
        first.resize(mark.size());
      }
      if (mark[(size_t)r] != calls) {
        mark[(size_t)r] = calls;
        acc[(size_t)r] = 0;
        first[(size_t)r] = j;
      }
      acc[(size_t)r] += c;
      rows[(size_t)j] = r;
    }
    std::vector<Py_ssize_t> out;
    std::vector<int64_t> hot;
    for (Py_ssize_t j = 0; j < m; ++j) {
      const int64_t r = rows[(size_t)j];
      if (r < 0 || first[(size_t)r] != j) continue;
      const int64_t sh = std::min<int64_t>(std::max<int64_t>(now - e[(size_t)r], 0), 62);
      const int64_t v = (u[(size_t)r] >> sh) + acc[(size_t)r];
      u[(size_t)r] = v;
      e[(size_t)r] = now;
      t[(size_t)r] = tick;
      if (v >= hot_at) {
        out.push_back(j);
        hot.push_back(r);
      }
    }
    ++tick;
    if (!hot.empty()) remove(hot);
    if (size() > cap) {  // the least recently counted, down to 7/8 of cap
      const size_t n = size(), drop = std::min(n, n - cap + cap / 8);
      std::vector<int64_t> order(n);
      for (size_t r = 0; r < n; ++r) order[r] = (int64_t)r;
      if (drop < n)  // (ties: the lower row first, as the array form's stable sort)
        std::nth_element(order.begin(), order.begin() + (Py_ssize_t)drop, order.end(), [&](int64_t a, int64_t b) {
          return t[(size_t)a] < t[(size_t)b] || (t[(size_t)a] == t[(size_t)b] && a < b);
        });
      order.resize(drop);
      remove(order);
    }
    return out;
  }
};
void use_table_free(PyObject* cap) { delete (UseTable*)PyCapsule_GetPointer(cap, "edv.usetable"); }
UseTable* use_table_of(PyObject* cap) { return (UseTable*)PyCapsule_GetPointer(cap, "edv.usetable"); }

PyObject* py_use_table(PyObject*, PyObject* args) {
  Py_ssize_t cap;
  if (!PyArg_ParseTuple(args, "n", &cap)) return nullptr;
  return PyCapsule_New(new UseTable((size_t)std::max<Py_ssize_t>(cap, 1)), "edv.usetable", use_table_free);
}

// use_table_add(table, flat, counts, floor, now, hot_at) -> bytes of int64 positions (UseTable::add);
// flat: 32 m bytes, counts: m int64
PyObject* py_use_table_add(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_buffer bk, bc;
  long long floor_, now, hot_at;
  if (!PyArg_ParseTuple(args, "Oy*y*LLL", &cap, &bk, &bc, &floor_, &now, &hot_at)) return nullptr;
  UseTable* ut = use_table_of(cap);
  PyObject* ret = nullptr;
  if (ut && bk.len % 32 == 0 && bc.len == bk.len / 4) {
    const std::vector<Py_ssize_t> out =
        ut->add((const char*)bk.buf, (const int64_t*)bc.buf, bk.len / 32, floor_, now, hot_at);
    std::vector<int64_t> o(out.begin(), out.end());
    ret = PyBytes_FromStringAndSize((const char*)o.data(), (Py_ssize_t)(8 * o.size()));
  } else if (ut) {
    PyErr_SetString(PyExc_ValueError, "use_table_add: 32-byte keys and one int64 count each");
  }
  PyBuffer_Release(&bk);
  PyBuffer_Release(&bc);
  return ret;
}

// use_table_pop(table, key32) -> (count, epoch) or None (the key's row freed)
PyObject* py_use_table_pop(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_buffer bk;
  if (!PyArg_ParseTuple(args, "Oy*", &cap, &bk)) return nullptr;
  UseTable* ut = use_table_of(cap);
  PyObject* ret = nullptr;
  if (ut && bk.len == 32) {
    uint64_t w[4];
    memcpy(w, bk.buf, 32);
    const int64_t r = ut->idx.get(w);
    if (r < 0) {
      ret = Py_None;
      Py_INCREF(ret);
    } else {
      ret = Py_BuildValue("(LL)", (long long)ut->u[(size_t)r], (long long)ut->e[(size_t)r]);
      std::vector<int64_t> gone{r};
      ut->remove(gone);
    }
  } else if (ut) {
    PyErr_SetString(PyExc_ValueError, "use_table_pop: a 32-byte key");
  }
  PyBuffer_Release(&bk);
  return ret;
}

PyObject* py_use_table_has(PyObject*, PyObject* args) {
  PyObject* cap;
  Py_buffer bk;
  if (!PyArg_ParseTuple(args, "Oy*", &cap, &bk)) return nullptr;
  UseTable* ut = use_table_of(cap);
  PyObject* ret = nullptr;
  if (ut) {
    uint64_t w[4] = {0, 0, 0, 0};
    if (bk.len == 32) memcpy(w, bk.buf, 32);
    ret = PyBool_FromLong(bk.len == 32 && ut->idx.get(w) >= 0);
  }
  PyBuffer_Release(&bk);
  return ret;
}

PyObject* py_use_table_len(PyObject*, PyObject* cap) {
  UseTable* ut = use_table_of(cap);
  if (!ut) return nullptr;
  return PyLong_FromSize_t(ut->size());
}

// general_items(uidx, is_gen, flat) -> (gen, keys): a mixed batch's general-path items -- gen = the
// positions i (uint32, ascending) whose distinct identifier uidx[i] has is_gen[uidx[i]] != 0, keys
// = flat's 32-byte key of each, in that order -- on the worker pool (numpy's mask, flatnonzero and
// row gather took ~1.2 ms for 60k of 250k items)
PyObject* py_general_items(PyObject*, PyObject* args) {
  Py_buffer bu, bg, bf;
  if (!PyArg_ParseTuple(args, "y*y*y*", &bu, &bg, &bf)) return nullptr;
  PyObject* ret = nullptr;
  const Py_ssize_t n = bu.len / 4, nu = bg.len;
  if (bu.len % 4 || bf.len != 32 * nu) {
    PyErr_SetString(PyExc_ValueError, "general_items: uint32 ids, one flag and one 32-byte key per identifier");
  } else {
    const uint32_t* ui = (const uint32_t*)bu.buf;
    const uint8_t* isg = (const uint8_t*)bg.buf;
    const char* flat = (const char*)bf.buf;
    const Py_ssize_t nc = (n + kScanChunk - 1) / kScanChunk;
    std::vector<Py_ssize_t> cnt((size_t)nc + 1, 0);
    std::atomic<bool> bad{false};
    const int t = n >= 32768 ? scan_threads(n, 0) : 1;
    run_chunks(n, t, [&](int, Py_ssize_t a, Py_ssize_t b) {
      Py_ssize_t c = 0;
      for (Py_ssize_t i = a; i < b; ++i) {
        const uint32_t u = ui[i];
        if (u >= (uint32_t)nu) {
          bad.store(true, std::memory_order_relaxed);
          continue;
        }
        c += isg[u] != 0;
      }
      cnt[(size_t)(a / kScanChunk) + 1] = c;
    });
    if (bad.load()) {
      PyErr_SetString(PyExc_ValueError, "general_items: an identifier id out of range");
    } else {
      for (size_t c = 1; c < cnt.size(); ++c) cnt[c] += cnt[c - 1];
      const Py_ssize_t m = cnt.back();
      PyObject* gen = PyBytes_FromStringAndSize(nullptr, 4 * m);
      PyObject* keys = gen ? PyBytes_FromStringAndSize(nullptr, 32 * m) : nullptr;
      if (keys) {
        uint32_t* go = (uint32_t*)PyBytes_AS_STRING(gen);
        char* ko = PyBytes_AS_STRING(keys);
        run_chunks(n, t, [&](int, Py_ssize_t a, Py_ssize_t b) {
          Py_ssize_t at = cnt[(size_t)(a / kScanChunk)];
          for (Py_ssize_t i = a; i < b; ++i) {
            const uint32_t u = ui[i];
            if (!isg[u]) continue;
            go[at] = (uint32_t)i;
            memcpy(ko + 32 * at, flat + 32 * (size_t)u, 32);
            ++at;
          }
        });
        ret = Py_BuildValue("(NN)", gen, keys);
      } else {
        Py_XDECREF(gen);
      }
    }
  }
  PyBuffer_Release(&bu);
  PyBuffer_Release(&bg);
  PyBuffer_Release(&bf);
  return ret;
}

PyObject* py_gather_items(PyObject*, PyObject* args) {
  Py_buffer bs, bm, bo, bi;
  Py_ssize_t stride = 64;
  if (!PyArg_ParseTuple(args, "y*y*y*y*|n", &bs, &bm, &bo, &bi, &stride)) return nullptr;
  const uint64_t* off = (const uint64_t*)bo.buf;
  const uint32_t* idx = (const uint32_t*)bi.buf;
  const Py_ssize_t n = bo.len / 8 - 1, k = bi.len / 4;
  bool ok = stride == 64 || stride == kSigSlot;
  std::string sig, msg;
  std::vector<uint64_t> o((size_t)k + 1, 0);
  if (ok) sig.assign((size_t)k * (size_t)stride, '\0');
  ok = ok && n >= 0 && bs.len >= n * stride;
  for (Py_ssize_t j = 0; j < k && ok; ++j) {
    const uint32_t i = idx[j];
    if ((Py_ssize_t)i >= n || off[i + 1] < off[i] || off[i + 1] > (uint64_t)bm.len) {
      ok = false;
      break;
    }
    memcpy(&sig[(size_t)j * stride], (const char*)bs.buf + (size_t)i * stride, (size_t)stride);
    msg.append((const char*)bm.buf + off[i], off[i + 1] - off[i]);
    o[(size_t)j + 1] = msg.size();
  }
  PyBuffer_Release(&bs);
  PyBuffer_Release(&bm);
  PyBuffer_Release(&bo);
  PyBuffer_Release(&bi);
  if (!ok) {
    PyErr_SetString(PyExc_ValueError, "gather_items: stride, index or offsets out of range");
    return nullptr;
  }
  return Py_BuildValue("(y#y#y#)", sig.data(), (Py_ssize_t)sig.size(), msg.data(), (Py_ssize_t)msg.size(),
                       (const char*)o.data(), (Py_ssize_t)(o.size() * 8));
}

// ------------------------------------------------------- the node's per-message path
// Node.verifySignature calls authenticate(req) once per client REQUEST and once per PROPAGATE
// (node.py:2294-2314), ~n times per request; with the verdicts already cached by the verify-ahead,
// that call must cost a few microseconds.  authn_key does authenticate()'s host steps up to the
// verkey lookup (client_authn.py:72-92) in one native call: the signature / identifier presence
// checks, b58decode(signature) and the signing serialization, returned as crypto_sign_open's input
// sm = sig || ser (nacl_wrappers.py:108) -- the verdict cache's key together with the verkey's
// bytes.  None whenever the reference would raise (or the bytes need Python): the caller then
// takes the per-message Python path, which raises the reference's exception.

PyObject* g_key_sig = nullptr;  // interned "signature" / "identifier"
PyObject* g_key_idr = nullptr;

bool intern_keys() {
  if (!g_key_sig) g_key_sig = PyUnicode_InternFromString("signature");
  if (!g_key_idr) g_key_idr = PyUnicode_InternFromString("identifier");
  return g_key_sig && g_key_idr;
}

// authn_key(msg, ignore) -> (identifier, sm) | None
PyObject* py_authn_key(PyObject*, PyObject* args) {
  PyObject *msg, *ignore;
  if (!PyArg_ParseTuple(args, "OO", &msg, &ignore)) return nullptr;
  if (!PyDict_CheckExact(msg)) Py_RETURN_NONE;
  if (!intern_keys()) return nullptr;
  PyObject* sv = PyDict_GetItemWithError(msg, g_key_sig);  // borrowed
  PyObject* iv = sv ? PyDict_GetItemWithError(msg, g_key_idr) : nullptr;
  if (!sv || !iv) {
    PyErr_Clear();
    Py_RETURN_NONE;  // missing (or a key compare raised): the Python path
  }
  if (!PyUnicode_CheckExact(sv) || !PyUnicode_IS_ASCII(sv) || PyUnicode_GET_LENGTH(sv) == 0 ||
      !PyUnicode_CheckExact(iv) || PyUnicode_GET_LENGTH(iv) == 0)
    Py_RETURN_NONE;
  static std::vector<uint8_t> sig;  // the GIL serialises calls
  if (!b58decode_raw(PyUnicode_1BYTE_DATA(sv), (size_t)PyUnicode_GET_LENGTH(sv), sig)) Py_RETURN_NONE;
  PyObject* ign = nullptr;
  if (ignore != Py_None) {
    ign = PySequence_Fast(ignore, "ignore must be a sequence");
    if (!ign) return nullptr;
  }
  static OutBuf ser;
  ser.clear();
  const bool ok = ser_obj(msg, 0, ign, ser);
  Py_XDECREF(ign);
  if (!ok) Py_RETURN_NONE;
  PyObject* sm = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(sig.size() + ser.size()));
  if (!sm) return nullptr;
  char* d = PyBytes_AS_STRING(sm);
  if (!sig.empty()) memcpy(d, sig.data(), sig.size());
  if (ser.size()) memcpy(d + sig.size(), ser.data(), ser.size());
  PyObject* r = PyTuple_Pack(2, iv, sm);
  Py_DECREF(sm);
  return r;
}

inline uint64_t mix64(uint64_t h, uint64_t v) {
  const unsigned __int128 p = (unsigned __int128)(h ^ v) * 0x9E3779B97F4A7C15ull;
  return (uint64_t)p ^ (uint64_t)(p >> 64);
}

uint64_t hash_bytes(uint64_t h, const uint8_t* p, size_t n) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v;
    memcpy(&v, p + i, 8);
    h = mix64(h, v);
  }
  uint64_t t = 0;
  if (i < n) memcpy(&t, p + i, n - i);
  return mix64(h, t ^ ((uint64_t)n << 56));
}

// distinct_sm(sig64, msgs, off, short, uidx, fast) -> ([item], [sm]): the items of a
// scan_batch_u (slot 64) with a distinct (identifier, sm = sig64 || msgs[off[i]:off[i+1]]), in
// order of first occurrence, and their sm bytes.  Items the scan left to Python (fast 0) and
// items whose sm is shorter than 64 bytes (short 1: crypto_sign_open rejects them, no key or GPU
// needed) are left out.  The verify-ahead batches a drain's n copies of each request with this:
// one verify per distinct signed message.
PyObject* py_distinct_sm(PyObject*, PyObject* args) {
  Py_buffer bs, bm, bo, bsh, bu, bf;
  if (!PyArg_ParseTuple(args, "y*y*y*y*y*y*", &bs, &bm, &bo, &bsh, &bu, &bf)) return nullptr;
  struct Rel {
    Py_buffer* b[6];
    ~Rel() {
      for (Py_buffer* x : b) PyBuffer_Release(x);
    }
  } rel{{&bs, &bm, &bo, &bsh, &bu, &bf}};
  const Py_ssize_t n = bf.len;
  if (bsh.len < n || bu.len < 4 * n || bo.len < 8 * (n + 1) || bs.len < 64 * n) {
    PyErr_SetString(PyExc_ValueError, "buffer sizes do not match");
    return nullptr;
  }
  const uint8_t* sig = (const uint8_t*)bs.buf;
  const uint8_t* msg = (const uint8_t*)bm.buf;
  const uint64_t* off = (const uint64_t*)bo.buf;
  const uint8_t* shortv = (const uint8_t*)bsh.buf;
  const uint32_t* uidx = (const uint32_t*)bu.buf;
  const uint8_t* fast = (const uint8_t*)bf.buf;
  for (Py_ssize_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) {
      PyErr_SetString(PyExc_ValueError, "offsets decrease");
      return nullptr;
    }
  if (n && off[n] > (uint64_t)bm.len) {
    PyErr_SetString(PyExc_ValueError, "offsets outside the message buffer");
    return nullptr;
  }
  size_t cap = 64;
  while (cap < 2 * (size_t)n) cap <<= 1;
  std::vector<int64_t> tab(cap, -1);
  std::vector<uint64_t> hv;
  std::vector<Py_ssize_t> pick;
  hv.reserve(64);
  for (Py_ssize_t i = 0; i < n; ++i) {
    if (!fast[i] || shortv[i]) continue;
    const uint64_t m0 = off[i], ml = off[i + 1] - off[i];
    const uint64_t h = hash_bytes(hash_bytes(0x51EDull ^ uidx[i], sig + 64 * i, 64), msg + m0, (size_t)ml);
    size_t s = (size_t)h & (cap - 1);
    for (;; s = (s + 1) & (cap - 1)) {
      const int64_t j = tab[s];
      if (j < 0) {
        tab[s] = (int64_t)pick.size();
        pick.push_back(i);
        hv.push_back(h);
        break;
      }
      const Py_ssize_t k = pick[(size_t)j];
      if (hv[(size_t)j] == h && uidx[k] == uidx[i] && off[k + 1] - off[k] == ml &&
          memcmp(sig + 64 * k, sig + 64 * i, 64) == 0 && memcmp(msg + off[k], msg + m0, (size_t)ml) == 0)
        break;  // a copy of item k
    }
  }
  PyObject* items = PyList_New((Py_ssize_t)pick.size());
  PyObject* sms = items ? PyList_New((Py_ssize_t)pick.size()) : nullptr;
  if (!sms) {
    Py_XDECREF(items);
    return nullptr;
  }
  for (size_t j = 0; j < pick.size(); ++j) {
    const Py_ssize_t i = pick[j];
    const uint64_t ml = off[i + 1] - off[i];
    PyObject* b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(64 + ml));
    PyObject* ix = b ? PyLong_FromSsize_t(i) : nullptr;
    if (!ix) {
      Py_XDECREF(b);
      Py_DECREF(items);
      Py_DECREF(sms);
      return nullptr;
    }
    memcpy(PyBytes_AS_STRING(b), sig + 64 * i, 64);
    if (ml) memcpy(PyBytes_AS_STRING(b) + 64, msg + off[i], (size_t)ml);
    PyList_SET_ITEM(items, (Py_ssize_t)j, ix);
    PyList_SET_ITEM(sms, (Py_ssize_t)j, b);
  }
  PyObject* r = PyTuple_Pack(2, items, sms);
  Py_DECREF(items);
  Py_DECREF(sms);
  return r;
}

PyMethodDef kMethods[] = {
    {"scan_batch", py_scan_batch, METH_VARARGS,
     "scan_batch(msgs, ignore, threads=0, out=None) -> (fast, idrs, sig64, msgbuf, off, short): authenticate()'s "
     "host steps for a batch.  out = [bytearray, bytearray]: sig64 / msgbuf are written into them (grown, never "
     "shrunk: slice to n * 64 and off[n] bytes) and returned"},
    {"verify_one", py_verify_one, METH_VARARGS,
     "verify_one(fn, ctx, sig64, key_id, msg) -> bool: edv_verify_one at address fn on context ctx"},
    {"keys_known_flat", py_keys_known_flat, METH_VARARGS,
     "keys_known_flat(clients, fast_keys, identifiers, field) -> (keys, holes, flat): keys_known on the "
     "worker pool, plus the 32-byte keys in one buffer"},
    {"key_index", py_key_index, METH_NOARGS, "key_index() -> a native 32-byte key -> int64 index"},
    {"key_index_set", py_key_index_set, METH_VARARGS, "key_index_set(index, keys32, ids_int64)"},
    {"key_index_del", py_key_index_del, METH_VARARGS, "key_index_del(index, keys32)"},
    {"key_index_clear", py_key_index_clear, METH_O, "key_index_clear(index)"},
    {"key_index_len", py_key_index_len, METH_O, "key_index_len(index)"},
    {"key_index_get", py_key_index_get, METH_VARARGS, "key_index_get(index, flat) -> int64 ids, -1 absent"},
    {"use_table", py_use_table, METH_VARARGS, "use_table(cap) -> native decayed use counts of 32-byte keys"},
    {"general_items", py_general_items, METH_VARARGS,
     "general_items(uidx_u32, is_gen_u8, flat_keys) -> (positions u32, their 32-byte keys)"},
    {"use_table_add", py_use_table_add, METH_VARARGS,
     "use_table_add(table, flat, counts_int64, floor, now, hot_at) -> int64 positions that reached hot_at"},
    {"use_table_pop", py_use_table_pop, METH_VARARGS, "use_table_pop(table, key32) -> (count, epoch) or None"},
    {"use_table_has", py_use_table_has, METH_VARARGS, "use_table_has(table, key32) -> bool"},
    {"use_table_len", py_use_table_len, METH_O, "use_table_len(table)"},
    {"keys_known", py_keys_known, METH_VARARGS,
     "keys_known(clients, fast_keys, identifiers, field) -> (keys, holes): the remembered key of each identifier "
     "whose clients entry still holds the remembered verkey, else None (holes: their positions)"},
    {"gather_spans", py_gather_spans, METH_VARARGS,
     "gather_spans(sig, msgbuf, spans_u64, idx_u32, stride=64) -> (sig_k, msg_k, off_k): gather_items for a staged "
     "batch's item spans (starts[n] then ends[n])"},
    {"kid_map", py_kid_map, METH_VARARGS,
     "kid_map(old, identifiers, ids_u32) -> map: identifier text -> key id (0xffffffff: none) for the staged "
     "scan's speculation (old: a kid_map to update in place, or None)"},
    {"kid_map_size", py_kid_map_size, METH_O, "kid_map_size(map) -> entries"},
    {"scan_batch_u", py_scan_batch_u, METH_VARARGS,
     "scan_batch_u(msgs, ignore, threads=0, out=None, slot=64) -> (fast, uidx_u32, uniq, sig, msgbuf, off, short): "
     "scan_batch with the identifiers as indices into the batch's distinct identifiers; slot=96: sig is n "
     "96-byte signature slots (edverify.h EDV_SIG_SLOT96: base58 text decoded on the GPU, or raw R||S); out "
     "items may be any writable buffers large enough (e.g. the engine's pinned host memory)"},
    {"pack_range", py_pack_range, METH_VARARGS,
     "pack_range(handle, lo, hi): write items [lo, hi) of a deferred scan_batch_u (defer=1 returns the handle as "
     "an 8th element) into its output buffers"},
    {"repack_spans", py_repack_spans, METH_VARARGS,
     "repack_spans(buf, spans) -> (msgs, off): a staged scan's messages laid out contiguously with offsets"},
    {"gather_u32", py_gather_u32, METH_VARARGS,
     "gather_u32(table, idx, out=None) -> buffer: table[idx[i]] (uint32); out: a bytearray to grow and reuse, or "
     "any writable buffer of len(idx) * 4 bytes or more (e.g. pinned memory); slice the result to len(idx) * 4"},
    {"results_ok", py_results_ok, METH_VARARGS,
     "results_ok(ok, short, uidx, uniq) -> (results, failed indices) of a steady-state batch"},
    {"results_from", py_results_from, METH_VARARGS,
     "results_from(codes_u8, uidx_u32, uniq) -> list: uniq[uidx[i]] where codes[i] == 1, else None"},
    {"gather_items", py_gather_items, METH_VARARGS,
     "gather_items(sig, msgbuf, off, idx_u32, stride=64) -> (sig, msgbuf, off) of the selected items"},
    {"serialize_for_signing", py_serialize_for_signing, METH_VARARGS,
     "serialize_for_signing(obj, ignore=None) -> bytes, or None for the Python path"},
    {"b58decode", py_b58decode, METH_O, "b58decode(str | bytes) -> bytes, or None for the Python path"},
    {"b58_len64", py_b58_len64, METH_O,
     "b58_len64(text) -> 1 if b58decode(text) is exactly 64 bytes, 0 if another length, -1 if not base58"},
    {"b58encode_rows", py_b58encode_rows, METH_VARARGS,
     "b58encode_rows(buf, width) -> list of b58encode(row) for each width-byte row (synthetic loads)"},
    {"pack_split64", py_pack_split64, METH_VARARGS,
     "pack_split64(sigs, sers) -> (sig64, msgs, off_u64le, short): crypto_sign_open's split at byte 64"},
    {"pack_sm", py_pack_sm, METH_VARARGS, "pack_sm(sigs, sers, keys) -> (sm, off_u64le, pk32)"},
    {"authn_key", py_authn_key, METH_VARARGS,
     "authn_key(msg, ignore) -> (identifier, sm = b58decode(signature) || serialization) or None for the Python "
     "path: authenticate()'s host steps before getVerkey (client_authn.py:72-92) in one call"},
    {"distinct_sm", py_distinct_sm, METH_VARARGS,
     "distinct_sm(sig64, msgs, off, short, uidx, fast) -> ([item], [sm]): scanned items with a distinct "
     "(identifier, sig || ser), first occurrences, and their sm bytes"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_hostpack",
                       "Native host packing for the GPU authenticator (see csrc/hostpack.cpp)", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__hostpack(void) { return PyModule_Create(&kModule); }
