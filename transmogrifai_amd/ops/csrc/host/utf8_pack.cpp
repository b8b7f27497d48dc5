// UTF-8 packing of a Python list of str / None straight from the str objects' code-point storage (PEP 393
// kinds 1 / 2 / 4) -- the input buffer of the native text cleaner and tokenizer (utils/text.py _encode_batch),
// without the per-string bytes objects and the join of `[s.encode("utf-8") for s in strings]`.
// Called through ctypes.PyDLL (the GIL is held). A list element that is not a str or None, or a str holding a
// lone surrogate (which str.encode("utf-8") rejects), returns -1 and the caller takes the Python path.
#include <Python.h>
#include <stdint.h>
#include <string.h>

namespace {

template <typename CH>
inline int64_t utf8_len_t(const CH* d, Py_ssize_t n) {
  int64_t b = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    const uint32_t c = d[i];
    b += 1 + (c >= 0x80) + (c >= 0x800) + (c >= 0x10000);
    if (sizeof(CH) > 1 && c >= 0xD800 && c <= 0xDFFF) return -1;
  }
  return b;
}

template <typename CH>
inline void utf8_put_t(const CH* d, Py_ssize_t n, uint8_t* o) {
  for (Py_ssize_t i = 0; i < n; ++i) {
    const uint32_t c = d[i];
    if (c < 0x80) {
      *o++ = (uint8_t)c;
    } else if (c < 0x800) {
      *o++ = (uint8_t)(0xC0 | (c >> 6));
      *o++ = (uint8_t)(0x80 | (c & 0x3F));
    } else if (c < 0x10000) {
      *o++ = (uint8_t)(0xE0 | (c >> 12));
      *o++ = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
      *o++ = (uint8_t)(0x80 | (c & 0x3F));
    } else {
      *o++ = (uint8_t)(0xF0 | (c >> 18));
      *o++ = (uint8_t)(0x80 | ((c >> 12) & 0x3F));
      *o++ = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
      *o++ = (uint8_t)(0x80 | (c & 0x3F));
    }
  }
}

inline int64_t utf8_len(PyObject* s) {
  const Py_ssize_t n = PyUnicode_GET_LENGTH(s);
  switch (PyUnicode_KIND(s)) {
    case PyUnicode_1BYTE_KIND:
      return PyUnicode_IS_ASCII(s) ? n : utf8_len_t(PyUnicode_1BYTE_DATA(s), n);
    case PyUnicode_2BYTE_KIND:
      return utf8_len_t(PyUnicode_2BYTE_DATA(s), n);
    default:
      return utf8_len_t(PyUnicode_4BYTE_DATA(s), n);
  }
}

inline void utf8_put(PyObject* s, uint8_t* o) {
  const Py_ssize_t n = PyUnicode_GET_LENGTH(s);
  switch (PyUnicode_KIND(s)) {
    case PyUnicode_1BYTE_KIND:
      if (PyUnicode_IS_ASCII(s)) {
        memcpy(o, PyUnicode_1BYTE_DATA(s), (size_t)n);
        return;
      }
      utf8_put_t(PyUnicode_1BYTE_DATA(s), n, o);
      return;
    case PyUnicode_2BYTE_KIND:
      utf8_put_t(PyUnicode_2BYTE_DATA(s), n, o);
      return;
    default:
      utf8_put_t(PyUnicode_4BYTE_DATA(s), n, o);
  }
}

}  // namespace

extern "C" {

// offs[0..n]: byte offsets of the items' UTF-8 encodings (None and "" -> empty); returns the total, or -1.
int64_t tmog_utf8_offsets(PyObject* list, int64_t* offs) {
  if (!PyList_Check(list)) return -1;
  const Py_ssize_t n = PyList_GET_SIZE(list);
  int64_t tot = 0;
  offs[0] = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* s = PyList_GET_ITEM(list, i);
    if (s != Py_None) {
      if (!PyUnicode_Check(s)) return -1;
      const int64_t b = utf8_len(s);
      if (b < 0) return -1;
      tot += b;
    }
    offs[i + 1] = tot;
  }
  return tot;
}

// the encodings themselves into out (offs from tmog_utf8_offsets on the same, unchanged list)
int tmog_utf8_copy(PyObject* list, const int64_t* offs, uint8_t* out) {
  if (!PyList_Check(list)) return -1;
  const Py_ssize_t n = PyList_GET_SIZE(list);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* s = PyList_GET_ITEM(list, i);
    if (s == Py_None) continue;
    if (!PyUnicode_Check(s)) return -1;
    utf8_put(s, out + offs[i]);
  }
  return 0;
}

}  // extern "C"
