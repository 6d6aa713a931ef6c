// hvae_io.hip -- host-side loader of the reference's processed-data artifacts.
//
// Reference: load_training_data + _build_matrix + get_user_indices_from_df (src/ml/train.py:153-193), i.e.
//   pd.read_csv(train.csv / val.csv), positives = rows with binary_rating == 1 (when the column exists),
//   csr_matrix((ones, (user_to_idx[user_id], item_to_idx[asin])), shape) -- duplicate pairs summed --, and the
//   users of the file in first-appearance order that the mappings know.
// Here one pass over the memory-mapped CSV (RFC 4180 quoting as pandas reads it: quoted fields may hold commas,
// doubled quotes and newlines) looks the two key columns up in hash maps built from the mappings' keys and
// counting-sorts the positives straight into canonical CSR (rows ascending, columns ascending within a row,
// duplicates summed), with no DataFrame and no COO matrix in between. Host code only (no GPU work).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "hvae_common.h"

namespace hvae {
namespace {

struct KeyMap {
  std::unordered_map<std::string_view, int64_t> m;
  bool build(const char* keys, int64_t len, int64_t n) {
    m.reserve((size_t)n * 2);
    int64_t i = 0, start = 0;
    for (int64_t p = 0; p <= len; ++p) {
      if (p == len || keys[p] == '\0') {
        if (i >= n) return false;
        m.emplace(std::string_view(keys + start, (size_t)(p - start)), i++);
        start = p + 1;
      }
    }
    return i == n;
  }
  int64_t find(std::string_view k) const {
    auto it = m.find(k);
    return it == m.end() ? -1 : it->second;
  }
};

// One CSV field starting at p (< end): its text (quotes removed; doubled quotes kept as a pair and marked in
// `esc`) and the position after its delimiter. *eol is set when the field ended its record.
struct Field {
  std::string_view text;
  bool esc;
};

inline const char* next_field(const char* p, const char* end, Field* f, bool* eol) {
  f->esc = false;
  if (p < end && *p == '"') {
    const char* s = ++p;
    while (p < end) {
      if (*p == '"') {
        if (p + 1 < end && p[1] == '"') { f->esc = true; p += 2; continue; }
        break;
      }
      ++p;
    }
    f->text = std::string_view(s, (size_t)(p - s));
    if (p < end) ++p;  // closing quote
    // skip to the delimiter (pandas tolerates nothing here either; be lenient)
    while (p < end && *p != ',' && *p != '\n' && *p != '\r') ++p;
  } else {
    const char* s = p;
    while (p < end && *p != ',' && *p != '\n' && *p != '\r') ++p;
    f->text = std::string_view(s, (size_t)(p - s));
  }
  *eol = true;
  if (p < end && *p == ',') { *eol = false; return p + 1; }
  if (p < end && *p == '\r') ++p;
  if (p < end && *p == '\n') ++p;
  return p;
}

std::string unescape(std::string_view v) {
  std::string s;
  s.reserve(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    s.push_back(v[i]);
    if (v[i] == '"' && i + 1 < v.size() && v[i + 1] == '"') ++i;
  }
  return s;
}

// pandas' numeric reading of binary_rating compared with 1 ("1", "1.0", " 1", "1e0" are 1; "", "nan" are not)
inline bool is_one(std::string_view v) {
  std::string s(v);
  char* e = nullptr;
  const double d = strtod(s.c_str(), &e);
  return e != s.c_str() && d == 1.0;
}

}  // namespace
}  // namespace hvae

using namespace hvae;

extern "C" int hvae_read_interactions(const char* csv_path, const char* user_keys, int64_t user_keys_len,
                                      int64_t n_users, const char* item_keys, int64_t item_keys_len, int64_t n_items,
                                      int positives_only, hvae_host_csr* out) {
  HVAE_REQUIRE(csv_path && user_keys && item_keys && out && n_users > 0 && n_items > 0 && n_users < INT32_MAX &&
                   n_items < INT32_MAX,
               "hvae_read_interactions: bad args");
  std::memset(out, 0, sizeof(*out));
  KeyMap um, im;
  HVAE_REQUIRE(um.build(user_keys, user_keys_len, n_users), "hvae_read_interactions: user key count mismatch");
  HVAE_REQUIRE(im.build(item_keys, item_keys_len, n_items), "hvae_read_interactions: item key count mismatch");
  const int fd = open(csv_path, O_RDONLY);
  HVAE_REQUIRE(fd >= 0, "hvae_read_interactions: cannot open %s", csv_path);
  struct stat st;
  fstat(fd, &st);
  const size_t size = (size_t)st.st_size;
  const char* base = size ? static_cast<const char*>(mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0)) : nullptr;
  close(fd);
  HVAE_REQUIRE(size == 0 || base != MAP_FAILED, "hvae_read_interactions: mmap failed");
  const char* p = base;
  const char* end = base + size;
  // header
  int c_user = -1, c_item = -1, c_bin = -1, ncol = 0;
  bool eol = size == 0;
  while (!eol && p < end) {
    Field f;
    p = next_field(p, end, &f, &eol);
    const std::string name = f.esc ? unescape(f.text) : std::string(f.text);
    if (name == "user_id") c_user = ncol;
    else if (name == "asin") c_item = ncol;
    else if (name == "binary_rating") c_bin = ncol;
    ++ncol;
  }
  if (c_user < 0 || c_item < 0) {
    if (base) munmap(const_cast<char*>(base), size);
    HVAE_FAIL(HVAE_ERR_ARG, "hvae_read_interactions: %s has no user_id / asin column", csv_path);
  }
  const bool filter = positives_only && c_bin >= 0;
  std::vector<int32_t> rows, cols;
  std::vector<uint8_t> seen((size_t)n_users, 0);
  std::vector<int64_t> users;
  int64_t bad_user = 0, bad_item = 0, line = 1;
  std::string bad_key;
  while (p < end) {
    if (*p == '\n' || *p == '\r') { ++p; continue; }  // blank line (pandas skips it)
    std::string_view uk, ik, bk;
    bool ue = false, ie = false;
    int c = 0;
    eol = false;
    while (!eol && p < end) {
      Field f;
      p = next_field(p, end, &f, &eol);
      if (c == c_user) { uk = f.text; ue = f.esc; }
      else if (c == c_item) { ik = f.text; ie = f.esc; }
      else if (c == c_bin) bk = f.text;
      ++c;
    }
    ++line;
    const int64_t u = ue ? um.find(unescape(uk)) : um.find(uk);
    if (u >= 0 && !seen[(size_t)u]) { seen[(size_t)u] = 1; users.push_back(u); }
    if (filter && !is_one(bk)) continue;
    const int64_t it = ie ? im.find(unescape(ik)) : im.find(ik);
    if (u < 0 || it < 0) {
      if (bad_user + bad_item == 0) bad_key = std::string(u < 0 ? uk : ik);
      bad_user += u < 0;
      bad_item += it < 0;
      continue;
    }
    rows.push_back((int32_t)u);
    cols.push_back((int32_t)it);
  }
  if (base) munmap(const_cast<char*>(base), size);
  HVAE_REQUIRE(bad_user + bad_item == 0,
               "hvae_read_interactions: %lld positive rows with a user and %lld with an item the mappings do not "
               "know (first: '%s'); the reference's _build_matrix cannot index them either",
               (long long)bad_user, (long long)bad_item, bad_key.c_str());
  // counting sort by row, then columns ascending within a row and duplicates summed
  const int64_t nnz_in = (int64_t)rows.size();
  std::vector<int64_t> rp((size_t)n_users + 1, 0);
  for (int64_t i = 0; i < nnz_in; ++i) ++rp[(size_t)rows[i] + 1];
  for (int64_t r = 0; r < n_users; ++r) rp[(size_t)r + 1] += rp[(size_t)r];
  std::vector<int32_t> ci((size_t)nnz_in);
  {
    std::vector<int64_t> fill(rp.begin(), rp.end() - 1);
    for (int64_t i = 0; i < nnz_in; ++i) ci[(size_t)fill[(size_t)rows[i]]++] = cols[i];
  }
  rows.clear(); rows.shrink_to_fit();
  cols.clear(); cols.shrink_to_fit();
  auto* row_ptr = static_cast<int64_t*>(malloc(sizeof(int64_t) * ((size_t)n_users + 1)));
  auto* col_idx = static_cast<int32_t*>(malloc(sizeof(int32_t) * std::max<size_t>((size_t)nnz_in, 1)));
  auto* vals = static_cast<float*>(malloc(sizeof(float) * std::max<size_t>((size_t)nnz_in, 1)));
  auto* uo = static_cast<int64_t*>(malloc(sizeof(int64_t) * std::max<size_t>(users.size(), 1)));
  HVAE_REQUIRE(row_ptr && col_idx && vals && uo, "hvae_read_interactions: out of host memory");
  int64_t nnz = 0;
  row_ptr[0] = 0;
  for (int64_t r = 0; r < n_users; ++r) {
    int32_t* b = ci.data() + rp[(size_t)r];
    int32_t* e = ci.data() + rp[(size_t)r + 1];
    std::sort(b, e);
    for (int32_t* q = b; q < e;) {
      int32_t* q2 = q;
      while (q2 < e && *q2 == *q) ++q2;
      col_idx[nnz] = *q;
      vals[nnz] = (float)(q2 - q);
      ++nnz;
      q = q2;
    }
    row_ptr[r + 1] = nnz;
  }
  std::copy(users.begin(), users.end(), uo);
  out->row_ptr = row_ptr;
  out->col_idx = col_idx;
  out->vals = vals;
  out->n_rows = n_users;
  out->n_cols = n_items;
  out->nnz = nnz;
  out->users = uo;
  out->n_users_seen = (int64_t)users.size();
  out->n_records = line - 1;
  return HVAE_OK;
}

extern "C" void hvae_host_csr_free(hvae_host_csr* c) {
  if (!c) return;
  free(c->row_ptr);
  free(c->col_idx);
  free(c->vals);
  free(c->users);
  std::memset(c, 0, sizeof(*c));
}
