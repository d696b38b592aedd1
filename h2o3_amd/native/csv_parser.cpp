// Native multi-threaded CSV parser (host C++).
//
// Re-design of water/parser/CsvParser.java + ParseSetup.java (type and
// header guessing) + ParseDataset.java (parallel parse, categorical domain
// merge).  The reference parses 4 MB chunks inside MRTasks and ships
// categorical dictionaries between nodes; here one process parses its files
// with a thread pool, then the Python side pushes the dense columns to HBM.
//
// Semantics kept from the reference:
//  * column types are guessed from a sample of rows (numeric / time / enum),
//    then fixed; a non-numeric token in a numeric column becomes NA;
//  * NA tokens: empty field plus user strings (default "NA" etc.);
//  * header auto-detection: first row all non-numeric while the sample has
//    numeric data below it;
//  * quoted fields (RFC 4180, doubled quotes) may contain separators/newlines.
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

enum Kind { K_NUM = 0, K_CAT = 1, K_TIME = 2, K_STR = 3 };

struct Column {
  std::string name;
  int kind = K_NUM;
  std::vector<double> num;        // K_NUM / K_TIME
  std::vector<int> codes;         // K_CAT
  std::vector<std::string> domain;
};

struct Result {
  std::vector<Column> cols;
  long long nrows = 0;
  std::string error;
};

struct Field {
  const char* p;
  size_t n;
  bool quoted;
};

static inline void unquote(const char* p, size_t n, std::string& out) {
  out.clear();
  for (size_t i = 0; i < n; ++i) {
    if (p[i] == '"' && i + 1 < n && p[i + 1] == '"') { out.push_back('"'); ++i; }
    else out.push_back(p[i]);
  }
}

// Tokenize one record starting at s (ends at e, exclusive, newline stripped).
static void split_record(const char* s, const char* e, char sep, char quote, std::vector<Field>& out) {
  out.clear();
  const char* p = s;
  while (true) {
    if (p < e && *p == quote) {
      const char* q = p + 1;
      const char* start = q;
      while (q < e) {
        if (*q == quote) {
          if (q + 1 < e && q[1] == quote) { q += 2; continue; }
          break;
        }
        ++q;
      }
      out.push_back({start, (size_t)(q - start), true});
      p = q + 1;
      while (p < e && *p != sep) ++p;
    } else {
      const char* q = p;
      while (q < e && *q != sep) ++q;
      const char* a = p;
      const char* b = q;
      while (a < b && (*a == ' ' || *a == '\t') && sep != ' ' && sep != '\t') ++a;
      while (b > a && (b[-1] == ' ' || b[-1] == '\t' || b[-1] == '\r') && sep != ' ' && sep != '\t') --b;
      if (b > a && b[-1] == '\r') --b;
      out.push_back({a, (size_t)(b - a), false});
      p = q;
    }
    if (p >= e) break;
    ++p;  // skip sep
    if (p == e) { out.push_back({p, 0, false}); break; }
  }
}

static inline bool parse_double(const char* p, size_t n, double& v) {
  if (n == 0) return false;
  const char* a = p;
  const char* b = p + n;
  if (*a == '+') ++a;
  auto r = std::from_chars(a, b, v);
  if (r.ec == std::errc() && r.ptr == b) return true;
  // inf / nan spellings
  std::string s(a, b);
  for (auto& c : s) c = (char)tolower(c);
  if (s == "inf" || s == "infinity") { v = (p[0] == '-') ? -INFINITY : INFINITY; return true; }
  if (s == "-inf" || s == "-infinity") { v = -INFINITY; return true; }
  return false;
}

static bool all_digits(const char* p, size_t n) {
  for (size_t i = 0; i < n; ++i) if (p[i] < '0' || p[i] > '9') return false;
  return n > 0;
}

// yyyy-mm-dd[ T]hh:mm:ss[.fff]  or  yyyy/mm/dd  -> ms since epoch (UTC)
static bool parse_time(const char* p, size_t n, double& ms) {
  if (n < 8 || n > 32) return false;
  int Y = 0, M = 0, D = 0, h = 0, mi = 0, s = 0, frac = 0, fd = 0;
  size_t i = 0;
  auto num = [&](int digits, int& out) -> bool {
    out = 0;
    for (int k = 0; k < digits; ++k) {
      if (i >= n || p[i] < '0' || p[i] > '9') return false;
      out = out * 10 + (p[i++] - '0');
    }
    return true;
  };
  if (!num(4, Y)) return false;
  if (i >= n || (p[i] != '-' && p[i] != '/')) return false;
  char ds = p[i++];
  if (!num(2, M)) return false;
  if (i >= n || p[i] != ds) return false;
  ++i;
  if (!num(2, D)) return false;
  if (i < n) {
    if (p[i] != ' ' && p[i] != 'T') return false;
    ++i;
    if (!num(2, h)) return false;
    if (i >= n || p[i] != ':') return false;
    ++i;
    if (!num(2, mi)) return false;
    if (i < n && p[i] == ':') {
      ++i;
      if (!num(2, s)) return false;
      if (i < n && p[i] == '.') {
        ++i;
        while (i < n && p[i] >= '0' && p[i] <= '9') { if (fd < 3) { frac = frac * 10 + (p[i] - '0'); ++fd; } ++i; }
        while (fd < 3) { frac *= 10; ++fd; }
      }
    }
    if (i < n && p[i] == 'Z') ++i;
    if (i != n) return false;
  }
  if (M < 1 || M > 12 || D < 1 || D > 31 || h > 23 || mi > 59 || s > 60) return false;
  // days from civil (Howard Hinnant)
  int y = Y - (M <= 2);
  int era = (y >= 0 ? y : y - 399) / 400;
  unsigned yoe = (unsigned)(y - era * 400);
  unsigned doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
  unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  long long days = (long long)era * 146097 + (long long)doe - 719468;
  ms = (double)(((days * 24 + h) * 60 + mi) * 60 + s) * 1000.0 + frac;
  return true;
}

struct Parser {
  char sep;
  char quote;
  int header;
  std::unordered_set<std::string> na;
  int nthreads;

  bool is_na(const Field& f) const {
    if (f.n == 0 && !f.quoted) return true;
    if (na.empty()) return false;
    return na.count(std::string(f.p, f.n)) > 0;
  }
};

}  // namespace

extern "C" {

void* h2o_csv_parse(const char** paths, int npaths, char sep, int header, const char** na_list, int nna,
                    char quote, int nthreads, int sample_rows) {
  auto* R = new Result();
  Parser P;
  P.sep = sep;
  P.quote = quote ? quote : '"';
  P.header = header;
  for (int i = 0; i < nna; ++i) P.na.insert(na_list[i]);
  P.nthreads = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  // ---- read files and find record boundaries (quote aware)
  std::vector<std::string> bufs(npaths);
  struct Rec { const char* s; const char* e; };
  std::vector<Rec> recs;
  std::vector<size_t> file_first_rec;
  for (int fi = 0; fi < npaths; ++fi) {
    FILE* f = fopen(paths[fi], "rb");
    if (!f) { R->error = std::string("cannot open ") + paths[fi]; return R; }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    bufs[fi].resize(sz);
    if (sz > 0 && fread(&bufs[fi][0], 1, sz, f) != (size_t)sz) { fclose(f); R->error = "read error"; return R; }
    fclose(f);
    const char* b = bufs[fi].data();
    const char* e = b + sz;
    file_first_rec.push_back(recs.size());
    const char* s = b;
    bool inq = false;
    for (const char* p = b; p < e; ++p) {
      char c = *p;
      if (c == P.quote) inq = !inq;
      else if (c == '\n' && !inq) {
        const char* end = p;
        if (end > s && end[-1] == '\r') --end;
        recs.push_back({s, end});
        s = p + 1;
      }
    }
    if (s < e) {
      const char* end = e;
      if (end > s && end[-1] == '\r') --end;
      recs.push_back({s, end});
    }
  }
  // drop blank records and comment-only lines
  {
    std::vector<Rec> r2;
    r2.reserve(recs.size());
    std::vector<size_t> newfirst;
    size_t fidx = 0;
    for (size_t i = 0; i < recs.size(); ++i) {
      while (fidx < file_first_rec.size() && file_first_rec[fidx] == i) { newfirst.push_back(r2.size()); ++fidx; }
      const Rec& r = recs[i];
      bool blank = true;
      for (const char* p = r.s; p < r.e; ++p) if (*p != ' ' && *p != '\t' && *p != '\r') { blank = false; break; }
      if (blank) continue;
      if (r.s < r.e && *r.s == '#') continue;
      r2.push_back(r);
    }
    while (fidx < file_first_rec.size()) { newfirst.push_back(r2.size()); ++fidx; }
    recs.swap(r2);
    file_first_rec.swap(newfirst);
  }
  if (recs.empty()) { R->nrows = 0; return R; }
  // ---- sample for header / types
  std::vector<Field> fl;
  int ncols = 0;
  size_t ns = std::min<size_t>(recs.size(), (size_t)std::max(sample_rows, 2));
  std::vector<std::vector<std::string>> sample;
  for (size_t i = 0; i < ns; ++i) {
    split_record(recs[i].s, recs[i].e, P.sep, P.quote, fl);
    ncols = std::max<int>(ncols, (int)fl.size());
    std::vector<std::string> row;
    std::string tmp;
    for (auto& f : fl) { unquote(f.p, f.n, tmp); row.push_back(P.is_na(f) ? std::string("\x01NA") : tmp); }
    sample.push_back(row);
  }
  auto isnum = [&](const std::string& s) { double v; return parse_double(s.data(), s.size(), v); };
  bool has_header;
  if (header == 1) has_header = true;
  else if (header == -1) has_header = false;
  else {
    bool first_all_str = true;
    for (auto& s : sample[0]) if (s == "\x01NA" || isnum(s)) { first_all_str = false; break; }
    bool later_num = false;
    for (size_t i = 1; i < sample.size() && !later_num; ++i)
      for (auto& s : sample[i]) if (s != "\x01NA" && isnum(s)) { later_num = true; break; }
    has_header = first_all_str && (later_num || sample.size() == 1);
    if (first_all_str && !later_num && sample.size() > 1) {
      // all-string data: header if the first row values never reappear
      bool dup = false;
      for (size_t j = 0; j < sample[0].size() && !dup; ++j)
        for (size_t i = 1; i < sample.size(); ++i)
          if (j < sample[i].size() && sample[i][j] == sample[0][j]) { dup = true; break; }
      has_header = !dup;
    }
  }
  R->cols.resize(ncols);
  for (int j = 0; j < ncols; ++j) {
    R->cols[j].name = (has_header && j < (int)sample[0].size() && sample[0][j] != "\x01NA") ? sample[0][j]
                                                                                            : ("C" + std::to_string(j + 1));
  }
  size_t s0 = has_header ? 1 : 0;
  for (int j = 0; j < ncols; ++j) {
    bool any = false, allnum = true, alltime = true;
    for (size_t i = s0; i < sample.size(); ++i) {
      if (j >= (int)sample[i].size()) continue;
      const std::string& s = sample[i][j];
      if (s == "\x01NA") continue;
      any = true;
      double v;
      if (!parse_double(s.data(), s.size(), v)) allnum = false;
      double ms;
      if (!parse_time(s.data(), s.size(), ms)) alltime = false;
    }
    R->cols[j].kind = !any ? K_NUM : (allnum ? K_NUM : (alltime ? K_TIME : K_CAT));
  }
  // records to parse: skip header rows of every file
  std::vector<char> skip(recs.size(), 0);
  if (has_header) {
    for (size_t fi = 0; fi < file_first_rec.size(); ++fi) {
      size_t r = file_first_rec[fi];
      if (r < recs.size()) skip[r] = 1;
    }
  }
  std::vector<size_t> rows;
  rows.reserve(recs.size());
  for (size_t i = 0; i < recs.size(); ++i) if (!skip[i]) rows.push_back(i);
  const long long N = (long long)rows.size();
  R->nrows = N;
  for (auto& c : R->cols) {
    if (c.kind == K_CAT) c.codes.assign(N, -1);
    else c.num.assign(N, NAN);
  }
  // ---- parallel parse
  int T = (int)std::min<long long>(P.nthreads, std::max<long long>(1, N / 1024));
  std::vector<std::vector<std::unordered_map<std::string, int>>> dicts(T, std::vector<std::unordered_map<std::string, int>>(ncols));
  std::vector<std::vector<std::vector<std::string>>> dict_order(T, std::vector<std::vector<std::string>>(ncols));
  auto work = [&](int t) {
    long long a = N * t / T, b = N * (t + 1) / T;
    std::vector<Field> ff;
    std::string tmp;
    for (long long r = a; r < b; ++r) {
      const Rec& rc = recs[rows[r]];
      split_record(rc.s, rc.e, P.sep, P.quote, ff);
      int m = std::min<int>((int)ff.size(), ncols);
      for (int j = 0; j < m; ++j) {
        const Field& f = ff[j];
        if (P.is_na(f)) continue;
        Column& c = R->cols[j];
        if (c.kind == K_NUM) {
          double v;
          if (f.quoted) { unquote(f.p, f.n, tmp); if (parse_double(tmp.data(), tmp.size(), v)) c.num[r] = v; }
          else if (parse_double(f.p, f.n, v)) c.num[r] = v;
        } else if (c.kind == K_TIME) {
          double ms;
          if (parse_time(f.p, f.n, ms)) c.num[r] = ms;
        } else {
          if (f.quoted) unquote(f.p, f.n, tmp); else tmp.assign(f.p, f.n);
          auto& d = dicts[t][j];
          auto it = d.find(tmp);
          int code;
          if (it == d.end()) {
            code = (int)d.size();
            d.emplace(tmp, code);
            dict_order[t][j].push_back(tmp);
          } else code = it->second;
          c.codes[r] = code;
        }
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  // ---- merge categorical dictionaries (first-seen order; Python sorts)
  for (int j = 0; j < ncols; ++j) {
    Column& c = R->cols[j];
    if (c.kind != K_CAT) continue;
    std::unordered_map<std::string, int> g;
    std::vector<std::vector<int>> remap(T);
    for (int t = 0; t < T; ++t) {
      remap[t].resize(dict_order[t][j].size());
      for (size_t k = 0; k < dict_order[t][j].size(); ++k) {
        const std::string& s = dict_order[t][j][k];
        auto it = g.find(s);
        int code;
        if (it == g.end()) { code = (int)c.domain.size(); g.emplace(s, code); c.domain.push_back(s); }
        else code = it->second;
        remap[t][k] = code;
      }
    }
    std::vector<std::thread> th2;
    for (int t = 0; t < T; ++t) {
      th2.emplace_back([&, t]() {
        long long a = N * t / T, b = N * (t + 1) / T;
        for (long long r = a; r < b; ++r) if (c.codes[r] >= 0) c.codes[r] = remap[t][c.codes[r]];
      });
    }
    for (auto& x : th2) x.join();
  }
  return R;
}

const char* h2o_csv_error(void* h) { return ((Result*)h)->error.c_str(); }
int h2o_csv_ncols(void* h) { return (int)((Result*)h)->cols.size(); }
long long h2o_csv_nrows(void* h) { return ((Result*)h)->nrows; }
const char* h2o_csv_name(void* h, int j) { return ((Result*)h)->cols[j].name.c_str(); }
int h2o_csv_kind(void* h, int j) { return ((Result*)h)->cols[j].kind; }
void h2o_csv_num(void* h, int j, double* out) {
  auto& v = ((Result*)h)->cols[j].num;
  if (!v.empty()) memcpy(out, v.data(), v.size() * sizeof(double));
}
void h2o_csv_codes(void* h, int j, int* out) {
  auto& v = ((Result*)h)->cols[j].codes;
  if (!v.empty()) memcpy(out, v.data(), v.size() * sizeof(int));
}
int h2o_csv_domain_size(void* h, int j) { return (int)((Result*)h)->cols[j].domain.size(); }
const char* h2o_csv_domain(void* h, int j, int k) { return ((Result*)h)->cols[j].domain[k].c_str(); }
void h2o_csv_free(void* h) { delete (Result*)h; }

}  // extern "C"
