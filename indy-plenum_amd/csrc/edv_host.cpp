// edv_host.cpp -- native host-side request preparation for the GPU verifier
// (SURVEY.md section 8f row f-1), as a CPython extension module `_edvhost`.
//
// Once verification runs on the GPU, the per-request Python work in front of it
// dominates (base58 of the signature 13.8 us, of the verkey
// 7.7 us, serialisation 5.8 us per request).  This module does that work in C++
// with the reference's exact semantics, and packs a whole batch into the
// C-ABI layout of include/edv.h in one call:
//
//   b58decode / b58encode   base58==1.0.0 as called on the hot path
//                           (plenum/server/client_authn.py:94,
//                            plenum/common/verifier.py:29-50)
//   serialize               common/serializers/signing_serializer.py:35-92
//                           (SigningSerializer.serialize, toBytes=True)
//   pack_open_batch         the positional sig||msg split of
//                           stp_core/crypto/nacl_wrappers.py:232-242 + packing
//   open_verify             pack_open_batch + the synchronous edv_verify_batch call
//
// Any input outside the fast path (non-ASCII base58 text, non-str dict keys,
// an invalid character, an unacceptable type, ...) returns NotImplemented so the
// Python restatement raises the reference's exact exception; the fast path
// never produces a different result, only the same one sooner.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

const char kAlphabet[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
int8_t g_index[256];

void init_index() {
  memset(g_index, -1, sizeof g_index);
  for (int i = 0; i < 58; i++) g_index[uint8_t(kAlphabet[i])] = int8_t(i);
}

// whitespace removed by str.rstrip() for an ASCII string (str.isspace on ASCII:
// \t \n \v \f \r, \x1c-\x1f, space) and by bytes.rstrip() (no \x1c-\x1f)
inline bool str_space(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }
inline bool bytes_space(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

// base58 text -> bytes (base58 1.0.0 b58decode).  false = not handled here.
// The magnitude is built in 32-bit limbs, five base-58 digits (58^5 < 2^32) per
// multiply-add pass.
bool b58_decode(const uint8_t* s, size_t n, bool is_str, std::string* out) {
  while (n && (is_str ? str_space(s[n - 1]) : bytes_space(s[n - 1]))) n--;
  size_t ones = 0;
  while (ones < n && s[ones] == '1') ones++;
  // b58decode_int strips trailing bytes-whitespace again (a no-op after the above
  // for str input; for bytes input it already happened)
  std::vector<uint32_t> limb;  // little-endian 32-bit limbs of the integer
  limb.reserve((n - ones) / 5 + 2);
  size_t i = ones;
  while (i < n) {
    uint32_t chunk = 0, mul = 1;
    for (int k = 0; k < 5 && i < n; k++, i++) {
      const int d = g_index[s[i]];
      if (d < 0) return false;
      chunk = chunk * 58u + uint32_t(d);
      mul *= 58u;
    }
    uint64_t carry = chunk;
    for (auto& l : limb) {
      const uint64_t v = uint64_t(l) * mul + carry;
      l = uint32_t(v);
      carry = v >> 32;
    }
    if (carry) limb.push_back(uint32_t(carry));
  }
  out->assign(ones, '\0');
  bool lead = true;  // to_bytes of the integer has no leading zero bytes
  for (size_t k = limb.size(); k-- > 0;)
    for (int b = 3; b >= 0; b--) {
      const char c = char(limb[k] >> (8 * b));
      if (lead && c == 0) continue;
      lead = false;
      out->push_back(c);
    }
  return true;
}

// bytes -> base58 text (base58 1.0.0 b58encode): big-endian 32-bit limbs,
// divided by 58^5 per pass (five digits at a time).
std::string b58_encode(const uint8_t* v, size_t n) {
  size_t zeros = 0;
  while (zeros < n && v[zeros] == 0) zeros++;
  const size_t len = n - zeros;
  std::vector<uint32_t> num((len + 3) / 4, 0);  // big-endian limbs
  for (size_t i = 0; i < len; i++) {
    const size_t pos = len - 1 - i;  // byte significance
    num[num.size() - 1 - pos / 4] |= uint32_t(v[zeros + i]) << (8 * (pos % 4));
  }
  std::string rev;  // digits, least significant first
  size_t first = 0;
  while (first < num.size()) {
    uint64_t rem = 0;
    for (size_t k = first; k < num.size(); k++) {
      const uint64_t cur = (rem << 32) | num[k];
      num[k] = uint32_t(cur / 656356768u);  // 58^5
      rem = cur % 656356768u;
    }
    while (first < num.size() && num[first] == 0) first++;
    for (int d = 0; d < 5; d++) {
      if (first >= num.size() && rem == 0) break;  // no leading zero digits
      rev.push_back(kAlphabet[rem % 58u]);
      rem /= 58u;
    }
  }
  std::string s(zeros, '1');
  s.append(rev.rbegin(), rev.rend());
  return s;
}

// (data, len, is_str) of a str (ASCII only) or bytes argument; false = other
bool text_arg(PyObject* o, const uint8_t** p, Py_ssize_t* n, bool* is_str) {
  if (PyUnicode_Check(o)) {
    if (PyUnicode_READY(o) < 0 || !PyUnicode_IS_ASCII(o)) return false;
    *p = reinterpret_cast<const uint8_t*>(PyUnicode_DATA(o));
    *n = PyUnicode_GET_LENGTH(o);
    *is_str = true;
    return true;
  }
  if (PyBytes_Check(o)) {
    *p = reinterpret_cast<const uint8_t*>(PyBytes_AS_STRING(o));
    *n = PyBytes_GET_SIZE(o);
    *is_str = false;
    return true;
  }
  return false;
}

// b58_decode for str text of at most 128 characters, into out[cap], with no
// heap allocation (the decode threads of auth_core_batch): same semantics as
// b58_decode(s, n, true, ...); returns the byte length, or -1 if the text is
// not handled here (invalid character, too long, result longer than cap).
int b58_decode_small(const uint8_t* s, size_t n, uint8_t* out, size_t cap) {
  while (n && str_space(s[n - 1])) n--;
  if (n > 128) return -1;
  size_t ones = 0;
  while (ones < n && s[ones] == '1') ones++;
  uint64_t limb[12];  // little-endian 64-bit limbs; 128 digits < 2^751
  size_t nl = 0;
  size_t i = ones;
  while (i < n) {  // ten base-58 digits (58^10 < 2^59) per multiply-add pass
    uint64_t chunk = 0, mul = 1;
    for (int k = 0; k < 10 && i < n; k++, i++) {
      const int d = g_index[s[i]];
      if (d < 0) return -1;
      chunk = chunk * 58u + uint64_t(d);
      mul *= 58u;
    }
    uint64_t carry = chunk;
    for (size_t l = 0; l < nl; l++) {
      const unsigned __int128 v = (unsigned __int128)limb[l] * mul + carry;
      limb[l] = uint64_t(v);
      carry = uint64_t(v >> 64);
    }
    if (carry) limb[nl++] = carry;
  }
  size_t len = ones;
  bool lead = true;
  uint8_t tmp[100];
  size_t tl = 0;
  for (size_t k = nl; k-- > 0;)
    for (int b = 7; b >= 0; b--) {
      const uint8_t c = uint8_t(limb[k] >> (8 * b));
      if (lead && c == 0) continue;
      lead = false;
      tmp[tl++] = c;
    }
  len += tl;
  if (len > cap) return -1;
  memset(out, 0, ones);
  memcpy(out + ones, tmp, tl);
  return int(len);
}

PyObject* py_b58decode(PyObject*, PyObject* arg) {
  const uint8_t* p;
  Py_ssize_t n;
  bool is_str;
  std::string out;
  if (!text_arg(arg, &p, &n, &is_str)) Py_RETURN_NOTIMPLEMENTED;
  if (is_str && n <= 128) {  // the allocation-free decoder the batch path uses
    uint8_t buf[128];
    const int len = b58_decode_small(p, size_t(n), buf, sizeof buf);
    if (len >= 0) return PyBytes_FromStringAndSize(reinterpret_cast<const char*>(buf), len);
  }
  if (!b58_decode(p, size_t(n), is_str, &out)) Py_RETURN_NOTIMPLEMENTED;
  return PyBytes_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

PyObject* py_b58encode(PyObject*, PyObject* arg) {
  const uint8_t* p;
  Py_ssize_t n;
  bool is_str;
  if (!text_arg(arg, &p, &n, &is_str)) Py_RETURN_NOTIMPLEMENTED;
  const std::string s = b58_encode(p, size_t(n));
  return PyBytes_FromStringAndSize(s.data(), Py_ssize_t(s.size()));
}

// ------------------------------------------------------------ SigningSerializer
// Appends serialize(obj, level) to out.  Returns 1 ok, 0 = not handled here
// (caller falls back to Python), -1 = Python error set.
int ser(PyObject* obj, int level, PyObject* ignore, std::string& out);

int append_str(PyObject* s, std::string& out) {
  Py_ssize_t n;
  const char* u = PyUnicode_AsUTF8AndSize(s, &n);
  if (!u) {  // e.g. lone surrogates: let the Python path raise the reference's error
    PyErr_Clear();
    return 0;
  }
  out.append(u, size_t(n));
  return 1;
}

int append_pystr(PyObject* o, std::string& out) {  // str(o)
  PyObject* s = PyObject_Str(o);
  if (!s) return -1;
  const int r = append_str(s, out);
  Py_DECREF(s);
  return r;
}

int ser(PyObject* obj, int level, PyObject* ignore, std::string& out) {
  if (Py_EnterRecursiveCall(" in SigningSerializer")) return -1;
  int r = 1;
  if (PyUnicode_Check(obj)) {
    r = append_str(obj, out);
  } else if (PyDict_Check(obj)) {
    // keys (minus the top-level ignore list), sorted; str keys only here.
    // Request dicts have a handful of keys: a stack buffer and an insertion
    // sort (no heap allocation per dict).
    struct Item {
      const char* k;  // UTF-8 of the key object ko
      size_t n;
      PyObject* ko;
      PyObject* v;
    };
    constexpr Py_ssize_t kStack = 16;
    Item stack_items[kStack];
    std::vector<Item> heap_items;
    const Py_ssize_t cap = PyDict_GET_SIZE(obj);
    Item* items = stack_items;
    if (cap > kStack) {
      heap_items.resize(size_t(cap));
      items = heap_items.data();
    }
    Py_ssize_t cnt = 0;
    const bool ign_set = ignore && PyAnySet_Check(ignore);
    PyObject *k, *v;
    Py_ssize_t pos = 0;
    while (r == 1 && PyDict_Next(obj, &pos, &k, &v)) {
      if (!PyUnicode_CheckExact(k)) { r = 0; break; }
      if (level == 0 && ignore) {
        const int c = ign_set ? PySet_Contains(ignore, k) : PySequence_Contains(ignore, k);
        if (c < 0) { r = -1; break; }
        if (c) continue;
      }
      Py_ssize_t n;
      const char* u = PyUnicode_AsUTF8AndSize(k, &n);
      if (!u) { PyErr_Clear(); r = 0; break; }
      if (cnt >= cap) { r = 0; break; }  // the dict grew under us: leave it to Python
      Py_INCREF(k);  // str() of a value may run Python code: hold keys and values
      Py_INCREF(v);
      // insertion sort by UTF-8 bytes (== code point order == Python's str sort)
      Py_ssize_t at = cnt++;
      while (at > 0) {
        const Item& p = items[at - 1];
        const int c = memcmp(p.k, u, p.n < size_t(n) ? p.n : size_t(n));
        if (c < 0 || (c == 0 && p.n <= size_t(n))) break;
        items[at] = p;
        at--;
      }
      items[at] = Item{u, size_t(n), k, v};
    }
    if (r == 1) {
      for (Py_ssize_t i = 0; r == 1 && i < cnt; i++) {
        if (i) out.push_back('|');
        out.append(items[i].k, items[i].n);
        out.push_back(':');
        r = ser(items[i].v, level + 1, nullptr, out);
      }
    }
    for (Py_ssize_t i = 0; i < cnt; i++) {
      Py_DECREF(items[i].ko);
      Py_DECREF(items[i].v);
    }
  } else if (PyList_Check(obj)) {
    const Py_ssize_t n = PyList_GET_SIZE(obj);
    for (Py_ssize_t i = 0; r == 1 && i < n; i++) {
      if (i) out.push_back(',');
      PyObject* it = PyList_GET_ITEM(obj, i);
      Py_INCREF(it);
      r = ser(it, level + 1, nullptr, out);
      Py_DECREF(it);
    }
  } else if (obj == Py_None) {
    // None -> ""
  } else if (obj == Py_True) {
    out += "True";
  } else if (obj == Py_False) {
    out += "False";
  } else if (PyLong_CheckExact(obj)) {
    int overflow = 0;
    const long long x = PyLong_AsLongLongAndOverflow(obj, &overflow);
    if (overflow || (x == -1 && PyErr_Occurred())) {
      PyErr_Clear();
      r = append_pystr(obj, out);
    } else {
      char buf[24];
      char* e = buf + sizeof buf;
      char* q = e;
      unsigned long long u = x < 0 ? 0ull - (unsigned long long)x : (unsigned long long)x;
      do { *--q = char('0' + u % 10); u /= 10; } while (u);
      if (x < 0) *--q = '-';
      out.append(q, size_t(e - q));
    }
  } else if (PyLong_Check(obj) || PyFloat_Check(obj)) {
    r = append_pystr(obj, out);  // str(x): repr for floats, __str__ of int subclasses
  } else {
    r = 0;  // not an acceptable type: the Python path raises the reference's error
  }
  Py_LeaveRecursiveCall();
  return r;
}

// serialize(obj, topLevelKeysToIgnore=None) -> bytes, or NotImplemented
PyObject* py_serialize(PyObject*, PyObject* args) {
  PyObject* obj;
  PyObject* ignore = Py_None;
  if (!PyArg_ParseTuple(args, "O|O", &obj, &ignore)) return nullptr;
  if (ignore != Py_None && !PySequence_Check(ignore) && !PyAnySet_Check(ignore)) Py_RETURN_NOTIMPLEMENTED;
  std::string out;
  const int r = ser(obj, 0, ignore == Py_None ? nullptr : ignore, out);
  if (r < 0) return nullptr;
  if (r == 0) Py_RETURN_NOTIMPLEMENTED;
  return PyBytes_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

// ----------------------------------------------------------------- batch pack
// pack_open_batch(items) with items a sequence of (sig: bytes, msg: bytes,
// pk: bytes(32)) -> (sigs, pks, msgs, offsets(uint64 LE bytes), index list) where
// only the items that reach the verifier are packed: crypto_sign_open of
// sig + msg splits positionally (sm[:64] / sm[64:]), and sm shorter than 64
// bytes rejects without a verify.  A key that is not 32 bytes -> ValueError.
struct OpenPack {
  std::string sigs, pks, msgs;
  std::vector<uint64_t> off{0};
  std::vector<Py_ssize_t> idx;  // items that reach the verifier
};
// 0 = packed, -1 = Python error set
static int pack_open(PyObject* seq, OpenPack& o) {
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  for (Py_ssize_t k = 0; k < n; k++) {
    PyObject* it = PySequence_Fast_GET_ITEM(seq, k);
    if (!PyTuple_Check(it) || PyTuple_GET_SIZE(it) != 3) {
      PyErr_SetString(PyExc_TypeError, "items must be (sig, msg, pk) tuples");
      return -1;
    }
    char *s, *m, *p;
    Py_ssize_t ls, lm, lp;
    if (PyBytes_AsStringAndSize(PyTuple_GET_ITEM(it, 0), &s, &ls) < 0 ||
        PyBytes_AsStringAndSize(PyTuple_GET_ITEM(it, 1), &m, &lm) < 0 ||
        PyBytes_AsStringAndSize(PyTuple_GET_ITEM(it, 2), &p, &lp) < 0)
      return -1;
    if (lp != 32) {
      PyErr_SetString(PyExc_ValueError, "public key must be 32 bytes");
      return -1;
    }
    if (ls + lm < 64) continue;  // crypto_sign_open: smlen < 64 rejects
    // sm = sig || msg; signature = sm[:64], message = sm[64:]
    if (ls == 64) {
      o.sigs.append(s, 64);
      o.msgs.append(m, size_t(lm));
    } else {
      std::string sm(s, size_t(ls));
      sm.append(m, size_t(lm));
      o.sigs.append(sm.data(), 64);
      o.msgs.append(sm.data() + 64, sm.size() - 64);
    }
    o.pks.append(p, 32);
    o.off.push_back(uint64_t(o.msgs.size()));
    o.idx.push_back(k);
  }
  o.msgs.append(64, '\0');  // the kernels read whole words past a message end
  return 0;
}

PyObject* py_pack_open_batch(PyObject*, PyObject* arg) {
  PyObject* seq = PySequence_Fast(arg, "pack_open_batch needs a sequence");
  if (!seq) return nullptr;
  OpenPack o;
  const int r = pack_open(seq, o);
  Py_DECREF(seq);
  if (r < 0) return nullptr;
  PyObject* idx = PyList_New(Py_ssize_t(o.idx.size()));
  if (!idx) return nullptr;
  for (size_t i = 0; i < o.idx.size(); i++) {
    PyObject* ki = PyLong_FromSsize_t(o.idx[i]);
    if (!ki) { Py_DECREF(idx); return nullptr; }
    PyList_SET_ITEM(idx, Py_ssize_t(i), ki);
  }
  return Py_BuildValue("(y#y#y#y#N)", o.sigs.data(), Py_ssize_t(o.sigs.size()), o.pks.data(),
                       Py_ssize_t(o.pks.size()), o.msgs.data(), Py_ssize_t(o.msgs.size()),
                       reinterpret_cast<const char*>(o.off.data()), Py_ssize_t(o.off.size() * 8), idx);
}

typedef int (*verify_fn_t)(const uint8_t*, const uint8_t*, const uint8_t*, const uint64_t*, uint64_t, uint8_t*,
                           uint32_t);

// open_verify(items, verify_addr, device_mask) -> list of bools, or the
// edv_verify_batch error code (an int) for the caller to raise on: pack_open_batch
// and the synchronous verify in one call, the GIL released around the device
// call (a Verifier.verify of one request spends no time in numpy or ctypes).
PyObject* py_open_verify(PyObject*, PyObject* args) {
  PyObject* items;
  unsigned long long vaddr;
  unsigned int mask;
  if (!PyArg_ParseTuple(args, "OKI", &items, &vaddr, &mask)) return nullptr;
  const verify_fn_t verify = reinterpret_cast<verify_fn_t>(uintptr_t(vaddr));
  PyObject* seq = PySequence_Fast(items, "open_verify needs a sequence");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  OpenPack o;
  const int r = pack_open(seq, o);
  Py_DECREF(seq);
  if (r < 0) return nullptr;
  const size_t nv = o.idx.size();
  std::vector<uint8_t> acc(nv ? nv : 1, 0);
  int rc = 0;
  if (nv) {
    Py_BEGIN_ALLOW_THREADS
    rc = verify(reinterpret_cast<const uint8_t*>(o.sigs.data()), reinterpret_cast<const uint8_t*>(o.pks.data()),
                reinterpret_cast<const uint8_t*>(o.msgs.data()), o.off.data(), uint64_t(nv), acc.data(), mask);
    Py_END_ALLOW_THREADS
  }
  if (rc != 0) return PyLong_FromLong(rc);
  PyObject* out = PyList_New(n);
  if (!out) return nullptr;
  for (Py_ssize_t k = 0; k < n; k++) {
    Py_INCREF(Py_False);
    PyList_SET_ITEM(out, k, Py_False);
  }
  for (size_t i = 0; i < nv; i++) {
    if (acc[i]) {
      Py_DECREF(Py_False);
      Py_INCREF(Py_True);
      PyList_SET_ITEM(out, o.idx[i], Py_True);
    }
  }
  return out;
}

// ------------------------------------------------------ CoreAuthNr fast path
// prep_core_batch(reqs, clients, excluded) -> list, one entry per request:
// (identifier, sig, ser, pk) when the request takes the common single-signature
// path of CoreAuthMixin.authenticate (plenum/server/client_authn.py:211-246) ->
// NaclAuthNr.authenticate_multi (:83-113) with SimpleAuthNr.getVerkey's
// in-memory `clients` map (:148-160) and DidVerifier (plenum/common/verifier.py:
// 26-52) yielding a 32-byte key; None otherwise (the Python plan handles that
// request, including every exception the reference would raise).
//   sig = b58decode(req["signature"])
//   ser = SigningSerializer bytes of req minus `excluded` (identifier present)
//   pk  = b58decode(idr) + b58decode(verkey[1:])  for a '~' abbreviated verkey
//         b58decode(verkey)                       otherwise
//         b58decode(idr)                          cryptonym: 32-byte idr, no verkey
bool b58_decode_obj(PyObject* o, std::string* out) {
  const uint8_t* p;
  Py_ssize_t n;
  bool is_str;
  return PyUnicode_CheckExact(o) && text_arg(o, &p, &n, &is_str) && b58_decode(p, size_t(n), is_str, out);
}

PyObject* prep_one_core(PyObject* req, PyObject* clients, PyObject* excluded) {
  if (!PyDict_CheckExact(req)) Py_RETURN_NONE;
  PyObject* idr = PyDict_GetItemString(req, "identifier");
  PyObject* sig = PyDict_GetItemString(req, "signature");
  if (!idr || !sig || !PyUnicode_CheckExact(idr) || !PyUnicode_CheckExact(sig) || PyUnicode_GET_LENGTH(idr) == 0 ||
      PyUnicode_GET_LENGTH(sig) == 0)
    Py_RETURN_NONE;
  std::string sigb, rawidr, pk;
  if (!b58_decode_obj(sig, &sigb)) Py_RETURN_NONE;
  PyObject* nym = PyDict_GetItemWithError(clients, idr);
  if (!nym) {
    if (PyErr_Occurred()) return nullptr;
    Py_RETURN_NONE;
  }
  if (!PyDict_CheckExact(nym) || PyDict_GET_SIZE(nym) == 0) Py_RETURN_NONE;
  PyObject* verkey = PyDict_GetItemString(nym, "verkey");
  if (!verkey || !PyUnicode_CheckExact(verkey)) Py_RETURN_NONE;
  if (!b58_decode_obj(idr, &rawidr)) Py_RETURN_NONE;
  const Py_ssize_t vl = PyUnicode_GET_LENGTH(verkey);
  if (vl == 0) {
    if (rawidr.size() != 32) Py_RETURN_NONE;  // ValueError / InvalidKey paths stay in Python
    pk = rawidr;                              // cryptonym
  } else if (PyUnicode_READ_CHAR(verkey, 0) == '~') {
    PyObject* abbr = PyUnicode_Substring(verkey, 1, vl);
    if (!abbr) return nullptr;
    std::string tail;
    const bool ok = b58_decode_obj(abbr, &tail);
    Py_DECREF(abbr);
    if (!ok) Py_RETURN_NONE;
    pk = rawidr + tail;  // b58decode(b58encode(x)) == x
  } else if (!b58_decode_obj(verkey, &pk)) {
    Py_RETURN_NONE;
  }
  if (pk.size() != 32) Py_RETURN_NONE;  // hex-encoded / empty keys: Python path
  std::string ser_out;
  const int r = ser(req, 0, excluded, ser_out);
  if (r < 0) return nullptr;
  if (r == 0) Py_RETURN_NONE;
  return Py_BuildValue("(Oy#y#y#)", idr, sigb.data(), Py_ssize_t(sigb.size()), ser_out.data(),
                       Py_ssize_t(ser_out.size()), pk.data(), Py_ssize_t(32));
}

PyObject* py_prep_core_batch(PyObject*, PyObject* args) {
  PyObject *reqs, *clients, *excluded;
  if (!PyArg_ParseTuple(args, "OO!O", &reqs, &PyDict_Type, &clients, &excluded)) return nullptr;
  PyObject* seq = PySequence_Fast(reqs, "prep_core_batch needs a sequence of requests");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject* out = PyList_New(n);
  if (!out) { Py_DECREF(seq); return nullptr; }
  for (Py_ssize_t k = 0; k < n; k++) {
    PyObject* e = prep_one_core(PySequence_Fast_GET_ITEM(seq, k), clients, excluded);
    if (!e) { Py_DECREF(out); Py_DECREF(seq); return nullptr; }
    PyList_SET_ITEM(out, k, e);
  }
  Py_DECREF(seq);
  return out;
}

// --------------------------------------------- whole-batch CoreAuthNr (f-1)
// auth_core_batch(reqs, clients, excluded, verify_addr, device_mask, threads[, resolved])
//   -> (out, slow, rejected)
// The single-signature fast path of prep_core_batch, done for a whole batch in
// one call with the GPU verify inside it:
//   phase A (GIL held)  type checks, verkey lookup (SimpleAuthNr.getVerkey,
//                       client_authn.py:148-160: the in-memory map, else the NYM
//                       the caller read from the uncommitted state, `resolved`),
//                       SigningSerializer bytes
//                       (client_authn.py:248-252) appended to the message arena;
//   phase B (no GIL)    base58 of signatures, identifiers and verkeys
//                       (client_authn.py:94, verifier.py:26-52) on `threads`
//                       threads, packed straight into the arena;
//   phase C (no GIL)    one call of the C-ABI verifier at verify_addr
//                       (edv_verify_batch, include/edv.h);
//   phase D (GIL held)  out[k] = [identifier] for an accepted request.
// slow: request indices outside the fast path (out[k] stays None; the caller's
// Python plan handles them, with every exception the reference raises);
// rejected: fast-path requests whose signature did not verify (the caller sets
// InsufficientCorrectSignatures(0, 1), the replay result of a failed single
// signature, client_authn.py:110-112).
typedef int (*host_alloc_t)(uint64_t, void**);
typedef int (*host_free_t)(void*);
host_alloc_t g_alloc = nullptr;
host_free_t g_free = nullptr;

// A reusable arena for one batch (page-locked through the library's
// edv_host_alloc when set_host_allocator was called, so the verifier DMAs it
// without a staging copy).  Only touched with the GIL held or by the call that
// owns it.
struct Arena {
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool pinned = false;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    release();
    bytes += bytes / 4 + 4096;
    void* q = nullptr;
    if (g_alloc && g_alloc(uint64_t(bytes), &q) == 0 && q) {
      pinned = true;
    } else {
      q = malloc(bytes);
      pinned = false;
      if (!q) return false;
    }
    p = static_cast<uint8_t*>(q);
    cap = bytes;
    return true;
  }
  void release() {
    if (p) {
      if (pinned && g_free) g_free(p);
      else if (!pinned) free(p);
    }
    p = nullptr;
    cap = 0;
  }
};
std::vector<Arena*> g_arenas;  // free list (GIL held)

Arena* take_arena() {
  if (g_arenas.empty()) return new Arena();
  Arena* a = g_arenas.back();
  g_arenas.pop_back();
  return a;
}

PyObject* py_set_host_allocator(PyObject*, PyObject* args) {
  unsigned long long a, f;
  if (!PyArg_ParseTuple(args, "KK", &a, &f)) return nullptr;
  for (Arena* x : g_arenas) { x->release(); delete x; }
  g_arenas.clear();
  g_alloc = reinterpret_cast<host_alloc_t>(uintptr_t(a));
  g_free = reinterpret_cast<host_free_t>(uintptr_t(f));
  Py_RETURN_NONE;
}

struct FastItem {
  Py_ssize_t k;
  PyObject *idr, *sig_o, *vk_o;  // referenced while the GIL is released (the decode reads their text)
  const uint8_t *sig, *idr_p, *vk_p;
  size_t sig_n, idr_n, vk_n;
  int vk_kind;  // 0 cryptonym (no verkey), 1 '~' abbreviated, 2 full verkey
};

inline bool ascii_str(PyObject* o, const uint8_t** p, size_t* n) {
  if (!PyUnicode_CheckExact(o) || PyUnicode_READY(o) < 0 || !PyUnicode_IS_ASCII(o)) return false;
  *p = reinterpret_cast<const uint8_t*>(PyUnicode_DATA(o));
  *n = size_t(PyUnicode_GET_LENGTH(o));
  return true;
}

// phase A for one request: false = not the fast path (nothing appended)
PyObject *g_k_identifier, *g_k_signature, *g_k_verkey;  // interned key strings (module init)
PyObject *g_k_reqid, *g_k_operation, *g_k_protocol, *g_k_type;

// verkey source of one identifier, as SimpleAuthNr.getVerkey (client_authn.py:148-160)
// reads it: the in-memory `clients` entry unless it is falsy, else the NYM the
// caller resolved from the uncommitted state (`resolved`: identifier -> nym dict,
// holding only non-empty dicts; None when the authenticator has no state).
// 1 = *nym set (a non-empty exact dict), 0 = not the fast path, -1 = error.
int lookup_nym(PyObject* clients, PyObject* resolved, PyObject* idr, PyObject** nym) {
  PyObject* v = PyDict_GetItemWithError(clients, idr);
  if (!v && PyErr_Occurred()) return -1;
  if (v && PyDict_CheckExact(v) && PyDict_GET_SIZE(v) > 0) { *nym = v; return 1; }
  // present but truthy and not a plain dict: the reference calls its .get (Python plan)
  if (v && v != Py_None && !(PyDict_CheckExact(v) && PyDict_GET_SIZE(v) == 0)) return 0;
  if (resolved == Py_None) return 0;
  v = PyDict_GetItemWithError(resolved, idr);
  if (!v) return PyErr_Occurred() ? -1 : 0;
  if (!PyDict_CheckExact(v) || PyDict_GET_SIZE(v) == 0) return 0;
  *nym = v;
  return 1;
}

// phase A for one request: 0 = not the fast path (nothing appended, no
// reference kept), 1 = *it filled and holding new references to idr, sig_o and
// vk_o (taken before ser(), which may run Python code: str() of an int
// subclass could otherwise drop the request's last reference to them), -1 = error.
int collect_one(PyObject* req, PyObject* clients, PyObject* resolved, PyObject* excluded, Py_ssize_t k,
                std::string& msgs, FastItem* it) {
  if (!PyDict_CheckExact(req)) return 0;
  PyObject* idr = PyDict_GetItem(req, g_k_identifier);
  PyObject* sig = PyDict_GetItem(req, g_k_signature);
  if (!idr || !sig) return 0;
  it->k = k;
  if (!ascii_str(sig, &it->sig, &it->sig_n) || !ascii_str(idr, &it->idr_p, &it->idr_n) || it->sig_n == 0 ||
      it->idr_n == 0)
    return 0;
  PyObject* nym = nullptr;
  const int lr = lookup_nym(clients, resolved, idr, &nym);
  if (lr <= 0) return lr;
  PyObject* verkey = PyDict_GetItem(nym, g_k_verkey);
  if (!verkey || !ascii_str(verkey, &it->vk_p, &it->vk_n)) return 0;
  if (it->vk_n == 0) {
    it->vk_kind = 0;
  } else if (it->vk_p[0] == '~') {
    it->vk_kind = 1;
    it->vk_p++;
    it->vk_n--;
  } else {
    it->vk_kind = 2;
  }
  Py_INCREF(idr);
  Py_INCREF(sig);
  Py_INCREF(verkey);
  it->idr = idr;
  it->sig_o = sig;
  it->vk_o = verkey;
  const size_t mark = msgs.size();
  const int r = ser(req, 0, excluded, msgs);
  if (r != 1) {
    msgs.resize(mark);
    Py_DECREF(idr);
    Py_DECREF(sig);
    Py_DECREF(verkey);
    return r;
  }
  return 1;
}

// phase B for one item: signature -> sig64, key -> pk32; false = not the fast path
bool decode_one(const FastItem& it, uint8_t* sig64, uint8_t* pk32) {
  uint8_t a[40], b[40];
  if (b58_decode_small(it.sig, it.sig_n, sig64, 64) != 64) return false;
  if (it.vk_kind == 2) return b58_decode_small(it.vk_p, it.vk_n, pk32, 32) == 32;
  const int la = b58_decode_small(it.idr_p, it.idr_n, a, sizeof a);
  if (la < 0) return false;
  if (it.vk_kind == 0) {
    if (la != 32) return false;  // cryptonym: the identifier is the key
    memcpy(pk32, a, 32);
    return true;
  }
  const int lb = b58_decode_small(it.vk_p, it.vk_n, b, sizeof b);
  if (lb < 0 || la + lb != 32) return false;
  memcpy(pk32, a, size_t(la));
  memcpy(pk32 + la, b, size_t(lb));
  return true;
}

double g_phase_s[4];  // seconds of the last auth_core_batch: A (GIL), B (decode), C (verify), D (output)
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
PyObject* py_last_phases(PyObject*, PyObject*) {
  return Py_BuildValue("{s:d,s:d,s:d,s:d}", "collect_serialize_s", g_phase_s[0], "decode_pack_s", g_phase_s[1],
                       "verify_s", g_phase_s[2], "output_s", g_phase_s[3]);
}

// The state of one whole-batch call between its phases (GIL held except where
// noted).  The item references and the arena are released by the destructor.
typedef int (*submit_fn_t)(const uint8_t*, const uint8_t*, const uint8_t*, const uint64_t*, uint64_t, uint8_t*,
                           uint8_t*, int, int64_t*);
typedef int (*wait_fn_t)(int, int64_t);
PyObject *g_k_signatures, *g_k_fees;

struct Batch {
  std::vector<FastItem> items;
  std::vector<Py_ssize_t> slow_idx;
  std::vector<uint8_t> good, dig_ok;  // per fast item: decoded; digest == sha256(signing bytes)
  std::string msgs;
  std::vector<uint64_t> moff = std::vector<uint64_t>(1, 0);
  Arena* ar = nullptr;
  size_t o_pk = 0, o_off = 0, o_msg = 0, o_acc = 0, o_dig = 0;
  Py_ssize_t n = 0;
  bool want_dig = false;
  // ReqAuthenticator mode (req_auth_submit): the batch's requests are todo[] of
  // n_all, kind[k] per request: 0 query, 1 no authenticator, 2 authenticated
  // here, 3 left to the general Python path
  bool req_mode = false;
  Py_ssize_t n_all = 0;
  std::vector<uint8_t> kind;
  std::vector<Py_ssize_t> todo;
  // asynchronous submission (auth_core_submit): the batch is in flight until waited for
  bool pending = false;
  // the wait for the device call failed: every later finish raises again (the
  // arena's verdict bytes are not the device's), and the arena is never reused
  // (a device slot may still reference it)
  bool failed = false;
  int device = 0;
  int64_t ticket = -1;
  wait_fn_t wait = nullptr;
  ~Batch() {
    for (FastItem& it : items) { Py_DECREF(it.idr); Py_DECREF(it.sig_o); Py_DECREF(it.vk_o); }
    if (ar && !failed) g_arenas.push_back(ar);  // failed: leaked on purpose
  }
};

// Wait for a submitted batch (GIL released).  0 = verdicts are in the arena;
// else the batch is marked failed, for good, and a Python error is set.
int finish_wait(Batch& b) {
  if (b.failed) {
    PyErr_SetString(PyExc_RuntimeError, "edv_wait_async failed earlier for this batch");
    return -1;
  }
  if (!b.pending) return 0;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = b.wait(b.device, b.ticket);
  Py_END_ALLOW_THREADS
  b.pending = false;
  if (rc != 0) {
    b.failed = true;
    PyErr_Format(PyExc_RuntimeError, "edv_wait_async failed (%d)", rc);
    return -1;
  }
  return 0;
}

// Request.getDigest (request.py:71-72) hashes the serialization of signingState =
// {identifier, reqId, operation[, protocolVersion if not None]} (request.py:77-87);
// the signing bytes serialize the request without signature / signatures / fees
// (client_authn.py:174, :222-223).  The two are the same bytes exactly when the
// request's other keys are identifier, reqId, operation and, unless it is None,
// protocolVersion.  -1 = error.
// Which of the request keys digest_is_signing_bytes cares about k is: 1
// signature / signatures / fees, 2 identifier / operation / reqId, 3
// protocolVersion, 0 any other.  Keys of a JSON-decoded request are equal to,
// not the same objects as, the interned names, so after the identity test one
// length switch and at most two memcmp (ASCII compact strings), not a chain of
// PyUnicode_CompareWithASCIIString calls per key.
int signing_key_kind(PyObject* k) {
  if (k == g_k_signature || k == g_k_signatures || k == g_k_fees) return 1;
  if (k == g_k_identifier || k == g_k_operation || k == g_k_reqid) return 2;
  if (k == g_k_protocol) return 3;
  if (PyUnicode_READY(k) < 0) {
    PyErr_Clear();
    return 0;
  }
  if (!PyUnicode_IS_COMPACT_ASCII(k)) return 0;  // none of the names
  const char* p = static_cast<const char*>(PyUnicode_DATA(k));
  auto eq = [p](const char* t, size_t n) { return memcmp(p, t, n) == 0; };
  switch (PyUnicode_GET_LENGTH(k)) {
    case 4: return eq("fees", 4) ? 1 : 0;
    case 5: return eq("reqId", 5) ? 2 : 0;
    case 9: return eq("signature", 9) ? 1 : (eq("operation", 9) ? 2 : 0);
    case 10: return eq("signatures", 10) ? 1 : (eq("identifier", 10) ? 2 : 0);
    case 15: return eq("protocolVersion", 15) ? 3 : 0;
    default: return 0;
  }
}

int digest_is_signing_bytes(PyObject* req) {
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  int have = 0;
  while (PyDict_Next(req, &pos, &k, &v)) {
    if (!PyUnicode_CheckExact(k)) return 0;
    switch (signing_key_kind(k)) {
      case 1: continue;
      case 2: have++; continue;
      case 3:
        if (v == Py_None) return 0;
        continue;
      default: return 0;  // any other key is in the signing bytes but not in signingState
    }
  }
  return have == 3 ? 1 : 0;
}

// phase A: collect, look verkeys up, serialize (GIL held)
int collect_all(Batch& b, PyObject* seq, PyObject* clients, PyObject* resolved, PyObject* excluded) {
  b.n = PySequence_Fast_GET_SIZE(seq);
  b.items.reserve(size_t(b.n));
  for (Py_ssize_t k = 0; k < b.n; k++) {
    PyObject* req = PySequence_Fast_GET_ITEM(seq, k);
    FastItem it;
    const int r = collect_one(req, clients, resolved, excluded, k, b.msgs, &it);
    if (r < 0) return -1;
    if (r == 0) { b.slow_idx.push_back(k); continue; }
    b.items.push_back(it);
    b.moff.push_back(uint64_t(b.msgs.size()));
    if (b.want_dig) {
      const int d = digest_is_signing_bytes(req);
      if (d < 0) return -1;
      b.dig_ok.push_back(uint8_t(d));
    }
  }
  return 0;
}

// A persistent pool for phase B: a Node's prod batch is a few hundred
// requests, for which starting threads per call would cost more than the
// decoding they share.  Workers never touch Python objects (they read the
// items' text, which the batch keeps referenced, and write the arena).
struct DecodePool {
  std::mutex mu;
  std::condition_variable go, done;
  int workers = 0, parts = 0, remaining = 0;
  uint64_t gen = 0;
  const std::function<void(int)>* job = nullptr;
  void ensure(int k) {  // caller holds no lock; called with the GIL held (one caller at a time)
    while (workers < k) {
      const int id = workers++;
      std::thread([this, id] { loop(id); }).detach();  // lives as long as the process
    }
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(mu);
        go.wait(lk, [&] { return gen != seen; });
        seen = gen;
        if (id + 1 >= parts) continue;
        f = job;
      }
      (*f)(id + 1);
      std::lock_guard<std::mutex> lk(mu);
      if (--remaining == 0) done.notify_all();
    }
  }
  // runs f(0..n-1): f(0) on the calling thread, the rest on workers
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 1) { f(0); return; }
    ensure(n - 1);
    {
      std::lock_guard<std::mutex> lk(mu);
      job = &f;
      parts = n;
      remaining = n - 1;
      gen++;
    }
    go.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [&] { return remaining == 0; });
  }
};
DecodePool* g_pool = nullptr;  // never destroyed: detached workers wait on it until exit
std::mutex g_pool_mu;          // one batch decodes at a time (the GIL is released meanwhile)

// phase B: arena + base58 decoding on `threads` threads (releases the GIL)
int pack_all(Batch& b, int threads) {
  const size_t nf = b.items.size();
  b.good.assign(nf, 1);
  if (!nf) return 0;
  b.ar = take_arena();
  // arena layout: sigs 64 nf | pks 32 nf | off 8 (nf + 1) | msgs (+64 slack) | accept nf | digests 32 nf
  b.o_pk = 64 * nf;
  b.o_off = b.o_pk + 32 * nf;
  b.o_msg = b.o_off + 8 * (nf + 1);
  b.o_acc = b.o_msg + ((b.msgs.size() + 64 + 63) / 64) * 64;
  b.o_dig = b.o_acc + ((nf + 63) / 64) * 64;
  if (!b.ar->ensure(b.o_dig + (b.want_dig ? 32 * nf : 0))) {
    PyErr_NoMemory();
    return -1;
  }
  uint8_t* base = b.ar->p;
  if (!g_pool) g_pool = new DecodePool();
  Py_BEGIN_ALLOW_THREADS
  // at least 1,024 requests per part: a Node prod's batch (a few hundred) decodes
  // on the calling thread, 0.40 us per request for submission and decode on the
  // MI355X box's host against 0.55-0.64 us with ~100-request parts on four
  // threads (the hand-offs cost more than the decoding they share,
  // profiles/r03/host_part_s22.log); only large batches spread out
  constexpr int kPart = 1024;
  const int T = std::max(1, std::min({threads, 32, int(nf / kPart)}));
  const std::function<void(int)> part = [&](int t) {
    const size_t lo = nf * size_t(t) / size_t(T), hi = nf * size_t(t + 1) / size_t(T);
    for (size_t i = lo; i < hi; i++)
      if (!decode_one(b.items[i], base + 64 * i, base + b.o_pk + 32 * i)) {
        b.good[i] = 0;
        memset(base + 64 * i, 0, 64);  // verified for nothing; the verdict is ignored
        memset(base + b.o_pk + 32 * i, 0, 32);
      }
    const size_t mlo = b.msgs.size() * size_t(t) / size_t(T), mhi = b.msgs.size() * size_t(t + 1) / size_t(T);
    memcpy(base + b.o_msg + mlo, b.msgs.data() + mlo, mhi - mlo);
  };
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool->run(T, part);
  }
  memcpy(base + b.o_off, b.moff.data(), 8 * (nf + 1));
  memset(base + b.o_msg + b.msgs.size(), 0, 64);
  memset(base + b.o_acc, 0, nf);  // reject until the device writes a verdict (arenas are reused)
  Py_END_ALLOW_THREADS
  return 0;
}

// phase D: (out, slow, rejected[, digests]).  For a large batch the cyclic GC
// is paused while the per-request lists are made: tens of thousands of new
// containers would otherwise trigger repeated collections that walk every live
// object of the node (30 ms per 64k batch, measured); the young objects are
// collected once, after.  A Node prod's batch (a few hundred requests) leaves
// the GC alone: pausing it would only move a collection that the node's own
// allocations made due to the first allocation after the pause, i.e. into the
// caller's authentication step (req_authenticator.GC_PAUSE_MIN, same bound).
constexpr Py_ssize_t kGcPauseMin = 4096;
inline int gc_pause_for(Py_ssize_t n) { return n >= kGcPauseMin ? PyGC_Disable() : 0; }

PyObject* build_output(Batch& b, bool with_digests) {
  const size_t nf = b.items.size();
  const uint8_t* acc = nf ? b.ar->p + b.o_acc : nullptr;
  const int gc_was = gc_pause_for(b.n);
  PyObject *out = PyList_New(b.n), *slow = PyList_New(0), *rejected = PyList_New(0), *digs = nullptr, *res = nullptr;
  if (with_digests) digs = PyList_New(b.n);
  if (!out || !slow || !rejected || (with_digests && !digs)) goto fail;
  for (Py_ssize_t k = 0; k < b.n; k++) {
    Py_INCREF(Py_None);
    PyList_SET_ITEM(out, k, Py_None);
    if (digs) {
      Py_INCREF(Py_None);
      PyList_SET_ITEM(digs, k, Py_None);
    }
  }
  for (Py_ssize_t k : b.slow_idx) {
    PyObject* v = PyLong_FromSsize_t(k);
    if (!v || PyList_Append(slow, v) < 0) { Py_XDECREF(v); goto fail; }
    Py_DECREF(v);
  }
  for (size_t i = 0; i < nf; i++) {
    const FastItem& it = b.items[i];
    if (digs && b.dig_ok[i]) {
      static const char hexd[] = "0123456789abcdef";
      const uint8_t* d = b.ar->p + b.o_dig + 32 * i;
      char h[64];
      for (int q = 0; q < 32; q++) {
        h[2 * q] = hexd[d[q] >> 4];
        h[2 * q + 1] = hexd[d[q] & 15];
      }
      PyObject* v = PyUnicode_FromStringAndSize(h, 64);
      if (!v) goto fail;
      PyObject* old = PyList_GET_ITEM(digs, it.k);
      PyList_SET_ITEM(digs, it.k, v);
      Py_DECREF(old);
    }
    if (!b.good[i]) {
      PyObject* v = PyLong_FromSsize_t(it.k);
      if (!v || PyList_Append(slow, v) < 0) { Py_XDECREF(v); goto fail; }
      Py_DECREF(v);
    } else if (acc[i]) {
      PyObject* l = PyList_New(1);
      if (!l) goto fail;
      Py_INCREF(it.idr);
      PyList_SET_ITEM(l, 0, it.idr);
      PyObject* old = PyList_GET_ITEM(out, it.k);
      PyList_SET_ITEM(out, it.k, l);
      Py_DECREF(old);
    } else {
      PyObject* v = PyLong_FromSsize_t(it.k);
      if (!v || PyList_Append(rejected, v) < 0) { Py_XDECREF(v); goto fail; }
      Py_DECREF(v);
    }
  }
  if (PyList_Sort(slow) < 0) goto fail;
  res = with_digests ? Py_BuildValue("(NNNN)", out, slow, rejected, digs) : Py_BuildValue("(NNN)", out, slow, rejected);
  if (gc_was) PyGC_Enable();
  return res;
fail:
  if (gc_was) PyGC_Enable();
  Py_XDECREF(out);
  Py_XDECREF(slow);
  Py_XDECREF(rejected);
  Py_XDECREF(digs);
  return nullptr;
}

bool parse_resolved(PyObject* resolved) {
  if (resolved != Py_None && !PyDict_Check(resolved)) {
    PyErr_SetString(PyExc_TypeError, "resolved must be a dict or None");
    return false;
  }
  return true;
}

PyObject* py_auth_core_batch(PyObject*, PyObject* args) {
  PyObject *reqs, *clients, *excluded, *resolved = Py_None;
  unsigned long long vaddr;
  unsigned int mask;
  int threads;
  if (!PyArg_ParseTuple(args, "OO!OKIi|O", &reqs, &PyDict_Type, &clients, &excluded, &vaddr, &mask, &threads,
                        &resolved) || !parse_resolved(resolved))
    return nullptr;
  const verify_fn_t verify = reinterpret_cast<verify_fn_t>(uintptr_t(vaddr));
  PyObject* seq = PySequence_Fast(reqs, "auth_core_batch needs a sequence of requests");
  if (!seq) return nullptr;
  Batch b;
  const double t0 = now_s();
  if (collect_all(b, seq, clients, resolved, excluded) < 0) { Py_DECREF(seq); return nullptr; }
  const double ta = now_s();
  if (pack_all(b, threads) < 0) { Py_DECREF(seq); return nullptr; }
  const double tb = now_s();
  int rc = 0;
  const size_t nf = b.items.size();
  if (nf) {
    uint8_t* base = b.ar->p;
    Py_BEGIN_ALLOW_THREADS
    // phase C: one device call
    rc = verify(base, base + b.o_pk, base + b.o_msg, reinterpret_cast<const uint64_t*>(base + b.o_off), uint64_t(nf),
                base + b.o_acc, mask);
    Py_END_ALLOW_THREADS
  }
  Py_DECREF(seq);
  if (rc != 0) {
    PyErr_Format(PyExc_RuntimeError, "edv_verify_batch failed (%d)", rc);
    return nullptr;
  }
  const double tc = now_s();
  PyObject* res = build_output(b, false);
  g_phase_s[0] = ta - t0;
  g_phase_s[1] = tb - ta;
  g_phase_s[2] = tc - tb;
  g_phase_s[3] = now_s() - tc;
  return res;
}

// ---- asynchronous whole batch (row f-2: the Node keeps going while the GPU works)
// auth_core_submit(reqs, clients, excluded, submit_addr, wait_addr, device, threads, resolved, want_digests)
//   -> handle: phases A and B as auth_core_batch, then ONE queued device call
//   (edv_verify_digest_batch_async at submit_addr) that returns at once;
// auth_core_finish(handle) -> (out, slow, rejected, digests or None): waits
//   (edv_wait_async at wait_addr, GIL released) and builds the lists.  With
//   want_digests, digests[k] is Request.getDigest() of request k when its signing
//   bytes are its signingState serialization (digest_is_signing_bytes), computed
//   on the device from the same bytes; None otherwise (the caller's digest path).
// A handle dropped unfinished waits for its batch before its arena is reused.
const char kBatchCapsule[] = "edv.auth_batch";

void batch_capsule_free(PyObject* cap) {
  Batch* b = static_cast<Batch*>(PyCapsule_GetPointer(cap, kBatchCapsule));
  if (!b) { PyErr_Clear(); return; }
  if (b->pending && b->wait) {
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = b->wait(b->device, b->ticket);  // the device may still write into the arena
    Py_END_ALLOW_THREADS
    if (rc != 0) b->failed = true;       // keep the arena out of the free list
  }
  delete b;
}

PyObject* py_auth_core_submit(PyObject*, PyObject* args) {
  PyObject *reqs, *clients, *excluded, *resolved = Py_None;
  unsigned long long saddr, waddr;
  int device, threads, want = 0;
  if (!PyArg_ParseTuple(args, "OO!OKKii|Op", &reqs, &PyDict_Type, &clients, &excluded, &saddr, &waddr, &device,
                        &threads, &resolved, &want) || !parse_resolved(resolved))
    return nullptr;
  PyObject* seq = PySequence_Fast(reqs, "auth_core_submit needs a sequence of requests");
  if (!seq) return nullptr;
  Batch* b = new Batch();
  b->want_dig = want != 0;
  b->device = device;
  b->wait = reinterpret_cast<wait_fn_t>(uintptr_t(waddr));
  PyObject* cap = PyCapsule_New(b, kBatchCapsule, batch_capsule_free);
  if (!cap) { delete b; Py_DECREF(seq); return nullptr; }
  if (collect_all(*b, seq, clients, resolved, excluded) < 0 || pack_all(*b, threads) < 0) {
    Py_DECREF(seq);
    Py_DECREF(cap);
    return nullptr;
  }
  Py_DECREF(seq);
  const size_t nf = b->items.size();
  if (!nf) return cap;
  const submit_fn_t submit = reinterpret_cast<submit_fn_t>(uintptr_t(saddr));
  uint8_t* base = b->ar->p;
  int64_t ticket = -1;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = submit(base, base + b->o_pk, base + b->o_msg, reinterpret_cast<const uint64_t*>(base + b->o_off),
              uint64_t(nf), base + b->o_acc, b->want_dig ? base + b->o_dig : nullptr, device, &ticket);
  Py_END_ALLOW_THREADS
  if (rc != 0) {
    Py_DECREF(cap);
    PyErr_Format(PyExc_RuntimeError, "edv_verify_digest_batch_async failed (%d)", rc);
    return nullptr;
  }
  b->ticket = ticket;
  b->pending = true;
  return cap;
}

PyObject* py_auth_core_finish(PyObject*, PyObject* cap) {
  Batch* b = static_cast<Batch*>(PyCapsule_GetPointer(cap, kBatchCapsule));
  if (!b) return nullptr;
  if (finish_wait(*b) < 0) return nullptr;
  if (b->want_dig) return build_output(*b, true);
  // (out, slow, rejected, None): the documented shape without digests too
  PyObject* r3 = build_output(*b, false);
  if (!r3) return nullptr;
  PyObject* r4 = Py_BuildValue("(OOOO)", PyTuple_GET_ITEM(r3, 0), PyTuple_GET_ITEM(r3, 1), PyTuple_GET_ITEM(r3, 2),
                               Py_None);
  Py_DECREF(r3);
  return r4;
}

// batch_ready(handle, query_addr) -> bool for an auth_core_submit or
// req_auth_submit handle: True when its finish will not wait for the device
// (the batch is done and its verdicts are in the arena, it failed -- finish
// raises -- or nothing was submitted), False while it is still on the GPU.
// query_addr: edv_query_async (EDV_PENDING = 1 while running).  Lets the Node
// hand a prod's batch over in the same prod when the GPU is already done.
typedef int (*query_fn_t)(int, int64_t);
PyObject* py_batch_ready(PyObject*, PyObject* args) {
  PyObject* cap;
  unsigned long long qaddr;
  if (!PyArg_ParseTuple(args, "OK", &cap, &qaddr)) return nullptr;
  Batch* b = static_cast<Batch*>(PyCapsule_GetPointer(cap, kBatchCapsule));
  if (!b) return nullptr;
  if (!b->pending || b->failed) Py_RETURN_TRUE;
  const query_fn_t query = reinterpret_cast<query_fn_t>(uintptr_t(qaddr));
  int rc;
  Py_BEGIN_ALLOW_THREADS  // the query takes the device's lock, which a synchronous call may hold
  rc = query(b->device, b->ticket);
  Py_END_ALLOW_THREADS
  if (rc == 1) Py_RETURN_FALSE;
  b->pending = false;
  if (rc != 0) b->failed = true;  // the finish raises, as after a failed wait (the arena is not reused)
  Py_RETURN_TRUE;
}

// ---- ReqAuthenticator.authenticate_batch_submit for the single stock
// CoreAuthNr (req_authenticator.py:22-44 per request): the txn-type routing too.
// req_auth_submit(reqs, clients, excluded, submit_addr, wait_addr, device, threads,
//                 resolved, want_digests, (query_types, write_types, action_types))
//   -> handle; kinds from req.get('operation', {}).get('type') against the three
//   type sets, exactly as the reference evaluates them; a request whose type
//   cannot be read that way (not a plain dict, an operation that is not a plain
//   dict, an unhashable type) is left to the general Python path.
// req_auth_finish(handle, NoAuthenticatorFound, InsufficientCorrectSignatures)
//   -> (out, slow, general, digests or None): out[k] is the set ReqAuthenticator
//   returns or the exception instance it raises; slow: requests the CoreAuthNr
//   Python plan must finish (its result r becomes r if an exception, else
//   set(r) or NoAuthenticatorFound()); general: requests for the general path.
PyObject* py_req_auth_submit(PyObject*, PyObject* args) {
  PyObject *reqs, *clients, *excluded, *resolved, *types;
  unsigned long long saddr, waddr;
  int device, threads, want;
  if (!PyArg_ParseTuple(args, "OO!OKKiiOpO!", &reqs, &PyDict_Type, &clients, &excluded, &saddr, &waddr, &device,
                        &threads, &resolved, &want, &PyTuple_Type, &types) || !parse_resolved(resolved))
    return nullptr;
  PyObject *qt, *wt, *at;
  if (!PyArg_ParseTuple(types, "OOO", &qt, &wt, &at)) return nullptr;
  PyObject* seq = PySequence_Fast(reqs, "req_auth_submit needs a sequence of requests");
  if (!seq) return nullptr;
  Batch* b = new Batch();
  b->req_mode = true;
  b->want_dig = want != 0;
  b->device = device;
  b->wait = reinterpret_cast<wait_fn_t>(uintptr_t(waddr));
  PyObject* cap = PyCapsule_New(b, kBatchCapsule, batch_capsule_free);
  if (!cap) { delete b; Py_DECREF(seq); return nullptr; }
  b->n_all = PySequence_Fast_GET_SIZE(seq);
  b->kind.assign(size_t(b->n_all), 3);
  PyObject* sub = PyList_New(0);
  if (!sub) { Py_DECREF(seq); Py_DECREF(cap); return nullptr; }
  for (Py_ssize_t k = 0; k < b->n_all; k++) {
    PyObject* req = PySequence_Fast_GET_ITEM(seq, k);
    if (!PyDict_CheckExact(req)) continue;  // general path
    PyObject* op = PyDict_GetItemWithError(req, g_k_operation);
    if (!op && PyErr_Occurred()) goto fail;
    PyObject* typ = Py_None;
    if (op) {
      if (!PyDict_CheckExact(op)) continue;
      typ = PyDict_GetItemWithError(op, g_k_type);
      if (!typ) {
        if (PyErr_Occurred()) goto fail;
        typ = Py_None;
      }
    }
    Py_INCREF(typ);  // the contains() calls below may run Python code
    int q = PySequence_Contains(qt, typ);
    int kd = -1;
    if (q > 0) kd = 0;
    else if (q == 0) {
      int w = PySequence_Contains(wt, typ);
      if (w == 0) w = PySequence_Contains(at, typ);
      if (w > 0) kd = 2;
      else if (w == 0) kd = 1;
    }
    Py_DECREF(typ);
    if (kd < 0) {
      PyErr_Clear();  // an unhashable type: the general path raises what the reference raises
      continue;
    }
    b->kind[size_t(k)] = uint8_t(kd);
    if (kd == 2) {
      b->todo.push_back(k);
      if (PyList_Append(sub, req) < 0) goto fail;
    }
  }
  Py_DECREF(seq);
  if (collect_all(*b, sub, clients, resolved, excluded) < 0 || pack_all(*b, threads) < 0) {
    Py_DECREF(sub);
    Py_DECREF(cap);
    return nullptr;
  }
  Py_DECREF(sub);
  {
    const size_t nf = b->items.size();
    if (!nf) return cap;
    const submit_fn_t submit = reinterpret_cast<submit_fn_t>(uintptr_t(saddr));
    uint8_t* base = b->ar->p;
    int64_t ticket = -1;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = submit(base, base + b->o_pk, base + b->o_msg, reinterpret_cast<const uint64_t*>(base + b->o_off),
                uint64_t(nf), base + b->o_acc, b->want_dig ? base + b->o_dig : nullptr, device, &ticket);
    Py_END_ALLOW_THREADS
    if (rc != 0) {
      Py_DECREF(cap);
      PyErr_Format(PyExc_RuntimeError, "edv_verify_digest_batch_async failed (%d)", rc);
      return nullptr;
    }
    b->ticket = ticket;
    b->pending = true;
  }
  return cap;
fail:
  Py_DECREF(sub);
  Py_DECREF(seq);
  Py_DECREF(cap);
  return nullptr;
}

PyObject* py_req_auth_finish(PyObject*, PyObject* args) {
  PyObject *cap, *no_auth, *ics;
  if (!PyArg_ParseTuple(args, "OOO", &cap, &no_auth, &ics)) return nullptr;
  Batch* b = static_cast<Batch*>(PyCapsule_GetPointer(cap, kBatchCapsule));
  if (!b) return nullptr;
  if (!b->req_mode) {
    PyErr_SetString(PyExc_TypeError, "not a req_auth_submit handle");
    return nullptr;
  }
  if (finish_wait(*b) < 0) return nullptr;
  const size_t nf = b->items.size();
  const uint8_t* acc = nf ? b->ar->p + b->o_acc : nullptr;
  const int gc_was = gc_pause_for(b->n_all);
  PyObject *out = PyList_New(b->n_all), *slow = PyList_New(0), *general = PyList_New(0), *digs = nullptr;
  PyObject* res = nullptr;
  if (b->want_dig) digs = PyList_New(b->n_all);
  if (!out || !slow || !general || (b->want_dig && !digs)) goto fail;
  for (Py_ssize_t k = 0; k < b->n_all; k++) {
    PyObject* v;
    switch (b->kind[size_t(k)]) {
      case 0: v = PySet_New(nullptr); break;                   // query: set()
      case 1: v = PyObject_CallNoArgs(no_auth); break;         // NoAuthenticatorFound
      case 3: {
        PyObject* i = PyLong_FromSsize_t(k);
        if (!i || PyList_Append(general, i) < 0) { Py_XDECREF(i); goto fail; }
        Py_DECREF(i);
      }  // fall through: placeholder None
      default: Py_INCREF(Py_None); v = Py_None;
    }
    if (!v) goto fail;
    PyList_SET_ITEM(out, k, v);
    if (digs) {
      Py_INCREF(Py_None);
      PyList_SET_ITEM(digs, k, Py_None);
    }
  }
  for (Py_ssize_t j : b->slow_idx) {  // collect-phase misses: CoreAuthNr's Python plan
    PyObject* i = PyLong_FromSsize_t(b->todo[size_t(j)]);
    if (!i || PyList_Append(slow, i) < 0) { Py_XDECREF(i); goto fail; }
    Py_DECREF(i);
  }
  for (size_t i = 0; i < nf; i++) {
    const FastItem& it = b->items[i];
    const Py_ssize_t k = b->todo[size_t(it.k)];
    if (digs && b->dig_ok[i]) {
      static const char hexd[] = "0123456789abcdef";
      const uint8_t* d = b->ar->p + b->o_dig + 32 * i;
      char h[64];
      for (int q = 0; q < 32; q++) {
        h[2 * q] = hexd[d[q] >> 4];
        h[2 * q + 1] = hexd[d[q] & 15];
      }
      PyObject* v = PyUnicode_FromStringAndSize(h, 64);
      if (!v) goto fail;
      PyObject* old = PyList_GET_ITEM(digs, k);
      PyList_SET_ITEM(digs, k, v);
      Py_DECREF(old);
    }
    PyObject* v = nullptr;
    if (!b->good[i]) {
      PyObject* ix = PyLong_FromSsize_t(k);
      if (!ix || PyList_Append(slow, ix) < 0) { Py_XDECREF(ix); goto fail; }
      Py_DECREF(ix);
      continue;
    } else if (acc[i]) {
      v = PySet_New(nullptr);                                  // {identifier}
      if (v && PySet_Add(v, it.idr) < 0) { Py_DECREF(v); v = nullptr; }
    } else {
      v = PyObject_CallFunction(ics, "ii", 0, 1);              // InsufficientCorrectSignatures(0, 1)
    }
    if (!v) goto fail;
    PyObject* old = PyList_GET_ITEM(out, k);
    PyList_SET_ITEM(out, k, v);
    Py_DECREF(old);
  }
  if (PyList_Sort(slow) < 0) goto fail;
  if (digs) res = Py_BuildValue("(NNNN)", out, slow, general, digs);
  else res = Py_BuildValue("(NNNO)", out, slow, general, Py_None);
  if (gc_was) PyGC_Enable();
  return res;
fail:
  if (gc_was) PyGC_Enable();
  Py_XDECREF(out);
  Py_XDECREF(slow);
  Py_XDECREF(general);
  Py_XDECREF(digs);
  return nullptr;
}

// ------------------------------------- state-backed verkeys (P5, rows f-1/f-3)
// state_nyms(reqs, clients, state_get, json_loads) -> {identifier: nym dict}
// SimpleAuthNr.getVerkey's second source (client_authn.py:148-160 ->
// domain_req_handler.py:158-167): for every distinct str identifier whose
// `clients` entry is missing or falsy, state_get(sha256(identifier), False)
// (nym_to_state_key; SHA-256 on the CPU here: one block per identifier), then
// the JSON value.  The usual value -- one flat object of plain strings, numbers,
// true/false/null -- is read here; anything else (escapes, nesting, non-ASCII,
// malformed text, a non-bytes value) goes to json_loads exactly as the Python
// restatement calls it.  Only non-empty objects are kept; for the fast-read ones
// the dict holds the one field the batch path reads ("verkey": str) and is left
// out when that is absent or not a string, so the Python plan raises what the
// reference raises for them.
#include "edv_sha256.h"

// Strict JSON subset scanner: 1 = parsed (vk/vk_n set if a string "verkey" was
// the last such key, *nkeys = member count), 0 = outside the subset.
int scan_flat_json(const uint8_t* p, size_t n, const uint8_t** vk, size_t* vk_n, bool* vk_str, int* nkeys) {
  size_t i = 0;
  auto ws = [&]() { while (i < n && (p[i] == ' ' || p[i] == '\t' || p[i] == '\n' || p[i] == '\r')) i++; };
  auto str = [&](const uint8_t** s, size_t* sn) -> bool {
    if (i >= n || p[i] != '"') return false;
    const size_t a = ++i;
    while (i < n && p[i] != '"') {
      if (p[i] < 0x20 || p[i] > 0x7e || p[i] == '\\') return false;
      i++;
    }
    if (i >= n) return false;
    *s = p + a;
    *sn = i - a;
    i++;
    return true;
  };
  auto digits = [&]() -> bool {
    const size_t a = i;
    while (i < n && p[i] >= '0' && p[i] <= '9') i++;
    return i > a;
  };
  auto number = [&]() -> bool {  // -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?
    if (i < n && p[i] == '-') i++;
    if (i >= n) return false;
    if (p[i] == '0') i++;
    else if (p[i] >= '1' && p[i] <= '9') digits();
    else return false;
    if (i < n && p[i] == '.') { i++; if (!digits()) return false; }
    if (i < n && (p[i] == 'e' || p[i] == 'E')) {
      i++;
      if (i < n && (p[i] == '+' || p[i] == '-')) i++;
      if (!digits()) return false;
    }
    return true;
  };
  auto lit = [&](const char* w) -> bool {
    const size_t k = strlen(w);
    if (i + k > n || memcmp(p + i, w, k) != 0) return false;
    i += k;
    return true;
  };
  *vk = nullptr;
  *vk_n = 0;
  *vk_str = false;
  *nkeys = 0;
  ws();
  if (i >= n || p[i] != '{') return 0;
  i++;
  ws();
  if (i < n && p[i] == '}') {
    i++;
  } else {
    for (;;) {
      const uint8_t* k;
      size_t kn;
      ws();
      if (!str(&k, &kn)) return 0;
      ws();
      if (i >= n || p[i] != ':') return 0;
      i++;
      ws();
      if (i >= n) return 0;
      const bool is_vk = kn == 6 && memcmp(k, "verkey", 6) == 0;
      if (p[i] == '"') {
        const uint8_t* v;
        size_t vn;
        if (!str(&v, &vn)) return 0;
        if (is_vk) { *vk = v; *vk_n = vn; *vk_str = true; }
      } else {
        const bool ok = (p[i] == 'n' && lit("null")) || (p[i] == 't' && lit("true")) ||
                        (p[i] == 'f' && lit("false")) || ((p[i] == '-' || (p[i] >= '0' && p[i] <= '9')) && number());
        if (!ok) return 0;
        if (is_vk) { *vk = nullptr; *vk_n = 0; *vk_str = false; }
      }
      (*nkeys)++;
      ws();
      if (i < n && p[i] == ',') { i++; continue; }
      if (i < n && p[i] == '}') { i++; break; }
      return 0;
    }
  }
  ws();
  return i == n ? 1 : 0;
}

// An ordinary exception raised for one identifier (not KeyboardInterrupt /
// SystemExit / MemoryError): cleared, and the identifier is left out.
bool skippable_error() {
  if (PyErr_ExceptionMatches(PyExc_Exception) && !PyErr_ExceptionMatches(PyExc_MemoryError)) {
    PyErr_Clear();
    return true;
  }
  return false;
}

PyObject* py_state_nyms(PyObject*, PyObject* args) {
  PyObject *reqs, *clients, *state_get, *json_loads;
  if (!PyArg_ParseTuple(args, "OO!OO", &reqs, &PyDict_Type, &clients, &state_get, &json_loads)) return nullptr;
  PyObject* seq = PySequence_Fast(reqs, "state_nyms needs a sequence of requests");
  if (!seq) return nullptr;
  PyObject* out = PyDict_New();
  PyObject* seen = PySet_New(nullptr);
  if (!out || !seen) { Py_XDECREF(out); Py_XDECREF(seen); Py_DECREF(seq); return nullptr; }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  std::vector<uint8_t> buf;
  for (Py_ssize_t k = 0; k < n; k++) {
    PyObject* req = PySequence_Fast_GET_ITEM(seq, k);
    if (!PyDict_CheckExact(req)) continue;
    PyObject* idr = PyDict_GetItem(req, g_k_identifier);
    if (!idr || !PyUnicode_CheckExact(idr) || PyUnicode_GET_LENGTH(idr) == 0) continue;
    const int s_in = PySet_Contains(seen, idr);
    if (s_in < 0) goto fail;
    if (s_in) continue;
    if (PySet_Add(seen, idr) < 0) goto fail;
    {
      PyObject* c = PyDict_GetItemWithError(clients, idr);
      if (!c && PyErr_Occurred()) goto fail;
      if (c) {
        const int t = PyObject_IsTrue(c);
        if (t < 0) goto fail;
        if (t) continue;  // getVerkey answers from the in-memory map
      }
    }
    Py_ssize_t ulen;
    const char* u = PyUnicode_AsUTF8AndSize(idr, &ulen);
    // an identifier that cannot be encoded (a lone surrogate is valid json.loads
    // output) or whose state read raises: skipped, so that request alone takes the
    // Python plan, whose getVerkey raises the reference's error for it alone
    if (!u) {
      if (!skippable_error()) goto fail;
      continue;
    }
    // nym_to_state_key: sha256(identifier.encode()), the kernel's SHA-256 on the CPU
    buf.assign(size_t(ulen) + 48, 0);
    memcpy(buf.data() + 16, u, size_t(ulen));
    uint32_t d[8];
    edv::sha256_msg(d, buf.data() + 16, uint64_t(ulen));
    uint8_t key[32];
    for (int w = 0; w < 8; w++) {
      key[4 * w] = uint8_t(d[w]);
      key[4 * w + 1] = uint8_t(d[w] >> 8);
      key[4 * w + 2] = uint8_t(d[w] >> 16);
      key[4 * w + 3] = uint8_t(d[w] >> 24);
    }
    PyObject* kb = PyBytes_FromStringAndSize(reinterpret_cast<const char*>(key), 32);
    if (!kb) goto fail;
    PyObject* data = PyObject_CallFunctionObjArgs(state_get, kb, Py_False, nullptr);
    Py_DECREF(kb);
    if (!data) {
      if (!skippable_error()) goto fail;
      continue;
    }
    const int truth = PyObject_IsTrue(data);
    if (truth <= 0) {
      Py_DECREF(data);
      if (truth < 0 && !skippable_error()) goto fail;
      continue;
    }
    const uint8_t* txt = nullptr;
    Py_ssize_t tn = 0;
    if (PyBytes_CheckExact(data)) {
      txt = reinterpret_cast<const uint8_t*>(PyBytes_AS_STRING(data));
      tn = PyBytes_GET_SIZE(data);
    } else if (PyUnicode_CheckExact(data) && PyUnicode_IS_ASCII(data)) {
      txt = reinterpret_cast<const uint8_t*>(PyUnicode_DATA(data));
      tn = PyUnicode_GET_LENGTH(data);
    }
    const uint8_t* vk;
    size_t vk_n;
    bool vk_str;
    int nkeys;
    PyObject* nym = nullptr;
    if (txt && scan_flat_json(txt, size_t(tn), &vk, &vk_n, &vk_str, &nkeys)) {
      if (nkeys > 0 && vk_str) {
        nym = PyDict_New();
        PyObject* v = nym ? PyUnicode_FromStringAndSize(reinterpret_cast<const char*>(vk), Py_ssize_t(vk_n)) : nullptr;
        if (!v || PyDict_SetItem(nym, g_k_verkey, v) < 0) { Py_XDECREF(v); Py_XDECREF(nym); Py_DECREF(data); goto fail; }
        Py_DECREF(v);
      }
    } else {
      // the Python restatement's exact call: json.loads(bytes(data).decode() or data)
      PyObject* arg = nullptr;
      if (PyBytes_Check(data) || PyByteArray_Check(data)) {
        arg = PyBytes_Check(data) ? PyUnicode_FromEncodedObject(data, "utf-8", "strict")
                                  : PyUnicode_DecodeUTF8(PyByteArray_AS_STRING(data), PyByteArray_GET_SIZE(data), "strict");
      } else {
        Py_INCREF(data);
        arg = data;
      }
      PyObject* v = arg ? PyObject_CallFunctionObjArgs(json_loads, arg, nullptr) : nullptr;
      Py_XDECREF(arg);
      if (!v) {
        PyErr_Clear();  // the reference raises here: the Python plan reproduces it
      } else if (PyDict_CheckExact(v) && PyDict_GET_SIZE(v) > 0) {
        nym = v;
      } else {
        Py_DECREF(v);
      }
    }
    Py_DECREF(data);
    if (nym) {
      const int rc = PyDict_SetItem(out, idr, nym);
      Py_DECREF(nym);
      if (rc < 0) goto fail;
    }
  }
  Py_DECREF(seen);
  Py_DECREF(seq);
  return out;
fail:
  Py_DECREF(out);
  Py_DECREF(seen);
  Py_DECREF(seq);
  return nullptr;
}

// ------------------------------------------------- request digests (f-3)
// request_digests(reqs, sha_addr, device_mask) -> list of hex str or None
// Request.getDigest() (plenum/common/request.py:71-72) for each request dict:
// sha256(serialize_msg_for_signing(signingState())).hexdigest(), signingState =
// {identifier, reqId, operation[, protocolVersion if not None]}
// (request.py:77-87).  Those four keys sort as identifier < operation <
// protocolVersion < reqId, so the serialization is written directly, without
// building the dict.  All messages go to one edv_sha256_batch call at sha_addr
// (GIL released).  None: a request this path does not handle (not a dict, no
// identifier -- the reference derives one from the signatures --, or a value
// the native serializer leaves to Python); the caller computes those in Python.
typedef int (*sha_fn_t)(const uint8_t*, const uint64_t*, uint64_t, uint8_t*, uint32_t);

PyObject* py_request_digests(PyObject*, PyObject* args) {
  PyObject* reqs;
  unsigned long long sha_addr;
  unsigned int mask;
  if (!PyArg_ParseTuple(args, "OKI", &reqs, &sha_addr, &mask)) return nullptr;
  PyObject* seq = PySequence_Fast(reqs, "request_digests needs a sequence");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  std::string msgs;
  msgs.reserve(size_t(n) * 160);
  std::vector<uint64_t> off(1, 0);
  std::vector<Py_ssize_t> where;  // request index of each hashed message
  where.reserve(size_t(n));
  for (Py_ssize_t k = 0; k < n; k++) {
    PyObject* r = PySequence_Fast_GET_ITEM(seq, k);
    if (!PyDict_Check(r)) continue;
    PyObject* idr = PyDict_GetItemWithError(r, g_k_identifier);
    if (!idr) {
      if (PyErr_Occurred()) { Py_DECREF(seq); return nullptr; }
      continue;
    }
    const int truth = PyObject_IsTrue(idr);
    if (truth < 0) { Py_DECREF(seq); return nullptr; }
    if (!truth) continue;
    PyObject* op = PyDict_GetItemWithError(r, g_k_operation);
    PyObject* rid = op || !PyErr_Occurred() ? PyDict_GetItemWithError(r, g_k_reqid) : nullptr;
    PyObject* pv = (op || !PyErr_Occurred()) && (rid || !PyErr_Occurred()) ? PyDict_GetItemWithError(r, g_k_protocol)
                                                                           : nullptr;
    if (PyErr_Occurred()) { Py_DECREF(seq); return nullptr; }
    const size_t mark = msgs.size();
    int rc = 1;
    msgs += "identifier:";
    rc = ser(idr, 1, nullptr, msgs);
    if (rc == 1) {
      msgs += "|operation:";
      if (op) rc = ser(op, 1, nullptr, msgs);
    }
    if (rc == 1 && pv && pv != Py_None) {
      msgs += "|protocolVersion:";
      rc = ser(pv, 1, nullptr, msgs);
    }
    if (rc == 1) {
      msgs += "|reqId:";
      if (rid) rc = ser(rid, 1, nullptr, msgs);
    }
    if (rc < 0) { Py_DECREF(seq); return nullptr; }
    if (rc == 0) {  // leave this one to Python
      msgs.resize(mark);
      continue;
    }
    off.push_back(uint64_t(msgs.size()));
    where.push_back(k);
  }
  const size_t m = where.size();
  std::vector<uint8_t> dig(32 * m);
  int rc = 0;
  if (m) {
    msgs.append(64, '\0');  // the kernel's tail loads may read past the last message
    sha_fn_t sha = reinterpret_cast<sha_fn_t>(sha_addr);
    Py_BEGIN_ALLOW_THREADS
    rc = sha(reinterpret_cast<const uint8_t*>(msgs.data()), off.data(), uint64_t(m), dig.data(), mask);
    Py_END_ALLOW_THREADS
  }
  Py_DECREF(seq);
  if (rc != 0) {
    PyErr_Format(PyExc_RuntimeError, "edv_sha256_batch failed (%d)", rc);
    return nullptr;
  }
  PyObject* out = PyList_New(n);
  if (!out) return nullptr;
  for (Py_ssize_t k = 0; k < n; k++) {
    Py_INCREF(Py_None);
    PyList_SET_ITEM(out, k, Py_None);
  }
  static const char hexd[] = "0123456789abcdef";
  for (size_t i = 0; i < m; i++) {
    char h[64];
    for (int b = 0; b < 32; b++) {
      h[2 * b] = hexd[dig[32 * i + b] >> 4];
      h[2 * b + 1] = hexd[dig[32 * i + b] & 15];
    }
    PyObject* v = PyUnicode_FromStringAndSize(h, 64);
    if (!v) { Py_DECREF(out); return nullptr; }
    PyObject* old = PyList_GET_ITEM(out, where[i]);
    PyList_SET_ITEM(out, where[i], v);
    Py_DECREF(old);
  }
  return out;
}

PyMethodDef kMethods[] = {
    {"auth_core_batch", py_auth_core_batch, METH_VARARGS,
     "whole-batch CoreAuthNr fast path with the GPU verify inside: (out, slow, rejected)"},
    {"last_phases", py_last_phases, METH_NOARGS, "phase seconds of the last auth_core_batch call"},
    {"state_nyms", py_state_nyms, METH_VARARGS,
     "NYMs of the identifiers getVerkey reads from the uncommitted state: {identifier: nym dict}"},
    {"auth_core_submit", py_auth_core_submit, METH_VARARGS,
     "asynchronous auth_core_batch (+ Request digests): queue the device call, return a handle"},
    {"req_auth_submit", py_req_auth_submit, METH_VARARGS,
     "ReqAuthenticator.authenticate_batch_submit for the single stock CoreAuthNr: type routing + auth_core_submit"},
    {"req_auth_finish", py_req_auth_finish, METH_VARARGS,
     "wait for a req_auth_submit handle: (out, slow, general, digests or None)"},
    {"auth_core_finish", py_auth_core_finish, METH_O,
     "wait for an auth_core_submit handle: (out, slow, rejected, digests or None)"},
    {"batch_ready", py_batch_ready, METH_VARARGS,
     "True when finishing a submitted handle will not wait for the device (edv_query_async at query_addr)"},
    {"set_host_allocator", py_set_host_allocator, METH_VARARGS,
     "page-locked arena allocator (edv_host_alloc, edv_host_free addresses)"},
    {"prep_core_batch", py_prep_core_batch, METH_VARARGS, "CoreAuthNr single-signature fast path (None = Python)"},
    {"b58decode", py_b58decode, METH_O, "base58 1.0.0 b58decode fast path (NotImplemented = use Python)"},
    {"b58encode", py_b58encode, METH_O, "base58 1.0.0 b58encode fast path (NotImplemented = use Python)"},
    {"serialize", py_serialize, METH_VARARGS, "SigningSerializer.serialize fast path (NotImplemented = use Python)"},
    {"request_digests", py_request_digests, METH_VARARGS,
     "Request.getDigest for a batch: one edv_sha256_batch call at sha_addr (None = use Python)"},
    {"pack_open_batch", py_pack_open_batch, METH_O, "pack (sig, msg, pk) items into the edv C-ABI layout"},
    {"open_verify", py_open_verify, METH_VARARGS, "crypto_sign_open verdicts of (sig, msg, pk) items, one device call"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_edvhost", "native host prep for the edv verifier", -1, kMethods,
                       nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__edvhost(void) {
  init_index();
  g_k_identifier = PyUnicode_InternFromString("identifier");
  g_k_signature = PyUnicode_InternFromString("signature");
  g_k_verkey = PyUnicode_InternFromString("verkey");
  g_k_reqid = PyUnicode_InternFromString("reqId");
  g_k_operation = PyUnicode_InternFromString("operation");
  g_k_protocol = PyUnicode_InternFromString("protocolVersion");
  g_k_signatures = PyUnicode_InternFromString("signatures");
  g_k_type = PyUnicode_InternFromString("type");
  g_k_fees = PyUnicode_InternFromString("fees");
  if (!g_k_identifier || !g_k_signature || !g_k_verkey) return nullptr;
  return PyModule_Create(&kModule);
}
