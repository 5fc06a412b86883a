/*
 * bloom_oracle.c — plain-C restatement of /root/reference/src/bloom.rs.
 * TEST INFRASTRUCTURE ONLY (see bloom_oracle.h): parity checker and CPU
 * baseline, never linked into the product library.
 */
#include "bloom_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

int ob_new(ob_filter* f, uint64_t m) {
  /* src/bloom.rs:17-21 — vec![false; size] */
  f->m = m;
  f->bits = NULL;
  if (m == 0) return OB_OK;
  f->bits = (uint8_t*)calloc(m, 1);
  return f->bits ? OB_OK : OB_ENOMEM;
}

void ob_free(ob_filter* f) {
  free(f->bits);
  f->bits = NULL;
  f->m = 0;
}

void ob_raw_hashes(const uint8_t* key, uint64_t len, uint64_t* h1o, uint64_t* h2o) {
  /* src/bloom.rs:28-34 — u64 wrapping arithmetic (unsigned overflow in C is
   * modulo 2^64, which is exactly Rust's wrapping_*). */
  uint64_t h1 = 5381, h2 = 0;
  for (uint64_t i = 0; i < len; ++i) {
    uint64_t b = key[i];
    h1 = ((h1 << 5) + h1) + b; /* (h1 << 5).wrapping_add(h1).wrapping_add(b) */
    h2 = h2 * 31u + b;         /* h2.wrapping_mul(31).wrapping_add(b) */
  }
  *h1o = h1;
  *h2o = h2;
}

int ob_hashes(const uint8_t* key, uint64_t len, uint64_t m, uint64_t* a, uint64_t* b) {
  uint64_t h1, h2;
  if (m == 0) return OB_EZEROM; /* src/bloom.rs:36 panics on % 0 */
  ob_raw_hashes(key, len, &h1, &h2);
  *a = h1 % m; /* src/bloom.rs:35-36 */
  *b = h2 % m;
  return OB_OK;
}

int ob_insert(ob_filter* f, const uint8_t* key, uint64_t len) {
  uint64_t a, b;
  int rc = ob_hashes(key, len, f->m, &a, &b);
  if (rc) return rc;
  f->bits[a] = 1; /* src/bloom.rs:42-43 */
  f->bits[b] = 1;
  return OB_OK;
}

int ob_may_contain(const ob_filter* f, const uint8_t* key, uint64_t len) {
  uint64_t a, b;
  int rc = ob_hashes(key, len, f->m, &a, &b);
  if (rc) return rc;
  /* src/bloom.rs:50 — `&&` short-circuits: bit b is only read if bit a is set */
  return f->bits[a] && f->bits[b];
}

int ob_insert_fixed(ob_filter* f, const uint8_t* keys, uint32_t key_len, uint64_t n) {
  if (n && f->m == 0) return OB_EZEROM;
  for (uint64_t i = 0; i < n; ++i) ob_insert(f, keys + i * (uint64_t)key_len, key_len);
  return OB_OK;
}

int ob_insert_var(ob_filter* f, const uint8_t* bytes, const uint64_t* off, uint64_t n) {
  if (n && f->m == 0) return OB_EZEROM;
  for (uint64_t i = 0; i < n; ++i) {
    if (off[i + 1] < off[i]) return OB_EINVAL;
    ob_insert(f, bytes + off[i], off[i + 1] - off[i]);
  }
  return OB_OK;
}

typedef struct {
  const ob_filter* const* fs;
  uint32_t nf;
  const uint8_t* bytes;
  const uint64_t* off; /* NULL for fixed-length keys */
  uint32_t key_len;
  uint64_t n, words, k0, k1;
  uint64_t* hits;
} probe_job;

static void* probe_range(void* arg) {
  probe_job* j = (probe_job*)arg;
  for (uint64_t k = j->k0; k < j->k1; ++k) {
    const uint8_t* key;
    uint64_t len;
    if (j->off) {
      key = j->bytes + j->off[k];
      len = j->off[k + 1] - j->off[k];
    } else {
      key = j->bytes + k * (uint64_t)j->key_len;
      len = j->key_len;
    }
    /* Database::get walks tables newest-first (src/lib.rs:130); the per-table
     * answer is independent of the order, so filters are visited 0..nf-1. */
    for (uint32_t f = 0; f < j->nf; ++f) {
      if (ob_may_contain(j->fs[f], key, len) == 1)
        j->hits[(uint64_t)f * j->words + (k >> 6)] |= (uint64_t)1 << (k & 63);
    }
  }
  return NULL;
}

static int probe_common(const ob_filter* const* fs, uint32_t nf, const uint8_t* bytes,
                        const uint64_t* off, uint32_t key_len, uint64_t n, uint64_t* hits,
                        int threads) {
  uint64_t words = (n + 63) / 64;
  for (uint32_t f = 0; f < nf; ++f)
    if (n && fs[f]->m == 0) return OB_EZEROM;
  if (off)
    for (uint64_t i = 0; i < n; ++i)
      if (off[i + 1] < off[i]) return OB_EINVAL;
  memset(hits, 0, (size_t)(words * nf * sizeof(uint64_t)));
  if (threads < 1) threads = 1;
  if ((uint64_t)threads > words) threads = words ? (int)words : 1;
  probe_job* jobs = (probe_job*)calloc((size_t)threads, sizeof(probe_job));
  pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  if (!jobs || !tids) {
    free(jobs);
    free(tids);
    return OB_ENOMEM;
  }
  /* ranges aligned to 64 keys so every hit word has exactly one writer */
  uint64_t per = ((words + threads - 1) / threads) * 64;
  for (int t = 0; t < threads; ++t) {
    probe_job* j = &jobs[t];
    j->fs = fs;
    j->nf = nf;
    j->bytes = bytes;
    j->off = off;
    j->key_len = key_len;
    j->n = n;
    j->words = words;
    j->hits = hits;
    j->k0 = per * t < n ? per * t : n;
    j->k1 = per * (t + 1) < n ? per * (t + 1) : n;
  }
  if (threads == 1) {
    probe_range(&jobs[0]);
  } else {
    for (int t = 0; t < threads; ++t) pthread_create(&tids[t], NULL, probe_range, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tids[t], NULL);
  }
  free(jobs);
  free(tids);
  return OB_OK;
}

int ob_probe_fixed(const ob_filter* const* fs, uint32_t nf, const uint8_t* keys,
                   uint32_t key_len, uint64_t n, uint64_t* hits, int threads) {
  return probe_common(fs, nf, keys, NULL, key_len, n, hits, threads);
}

int ob_probe_var(const ob_filter* const* fs, uint32_t nf, const uint8_t* bytes,
                 const uint64_t* offsets, uint64_t n, uint64_t* hits, int threads) {
  return probe_common(fs, nf, bytes, offsets, 0, n, hits, threads);
}

/* ---- prost codec for `message BloomProto { repeated bool bits = 1; }` ---- */

static uint64_t varint_len(uint64_t v) {
  uint64_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

static uint8_t* put_varint(uint8_t* p, uint64_t v) {
  while (v >= 0x80) {
    *p++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *p++ = (uint8_t)v;
  return p;
}

uint64_t ob_encode(const ob_filter* f, uint8_t* out, uint64_t cap) {
  /* prost encodes proto3 repeated scalars packed and omits empty fields */
  if (f->m == 0) return 0;
  uint64_t total = 1 + varint_len(f->m) + f->m;
  if (out && cap >= total) {
    uint8_t* p = out;
    *p++ = 0x0A; /* field 1, wire type 2 (length-delimited) */
    p = put_varint(p, f->m);
    for (uint64_t i = 0; i < f->m; ++i) p[i] = f->bits[i] ? 1 : 0;
  }
  return total;
}

/* prost's decode_varint: at most 10 bytes, the 10th must be <= 1. */
static int get_varint(const uint8_t** pp, const uint8_t* end, uint64_t* v) {
  const uint8_t* p = *pp;
  uint64_t r = 0;
  for (int i = 0; i < 10; ++i) {
    if (p >= end) return OB_EDECODE;
    uint8_t b = *p++;
    if (i == 9 && b > 1) return OB_EDECODE;
    r |= (uint64_t)(b & 0x7F) << (7 * i);
    if (!(b & 0x80)) {
      *pp = p;
      *v = r;
      return OB_OK;
    }
  }
  return OB_EDECODE;
}

typedef struct {
  uint8_t* v;
  uint64_t n, cap;
} bvec;

static int bvec_push(bvec* b, uint8_t x) {
  if (b->n == b->cap) {
    uint64_t nc = b->cap ? b->cap * 2 : 64;
    uint8_t* nv = (uint8_t*)realloc(b->v, nc);
    if (!nv) return OB_ENOMEM;
    b->v = nv;
    b->cap = nc;
  }
  b->v[b->n++] = x;
  return OB_OK;
}

static int skip_field(const uint8_t** pp, const uint8_t* end, uint32_t wt, uint64_t field,
                      int depth);

static int skip_group(const uint8_t** pp, const uint8_t* end, uint64_t field, int depth) {
  if (depth > 100) return OB_EDECODE; /* prost's recursion limit */
  for (;;) {
    uint64_t key;
    if (get_varint(pp, end, &key)) return OB_EDECODE;
    uint32_t wt = (uint32_t)(key & 7);
    uint64_t fn = key >> 3;
    if (fn == 0 || key > 0xFFFFFFFFull) return OB_EDECODE;
    if (wt == 4) return fn == field ? OB_OK : OB_EDECODE;
    if (skip_field(pp, end, wt, fn, depth + 1)) return OB_EDECODE;
  }
}

static int skip_field(const uint8_t** pp, const uint8_t* end, uint32_t wt, uint64_t field,
                      int depth) {
  uint64_t v;
  switch (wt) {
    case 0:
      return get_varint(pp, end, &v);
    case 1:
      if ((uint64_t)(end - *pp) < 8) return OB_EDECODE;
      *pp += 8;
      return OB_OK;
    case 2:
      if (get_varint(pp, end, &v)) return OB_EDECODE;
      if (v > (uint64_t)(end - *pp)) return OB_EDECODE;
      *pp += v;
      return OB_OK;
    case 3:
      return skip_group(pp, end, field, depth);
    case 5:
      if ((uint64_t)(end - *pp) < 4) return OB_EDECODE;
      *pp += 4;
      return OB_OK;
    default:
      return OB_EDECODE; /* 4 (unmatched end group), 6, 7 */
  }
}

int ob_decode(const uint8_t* in, uint64_t len, ob_filter* out) {
  const uint8_t* p = in;
  const uint8_t* end = in + len;
  bvec bits = {NULL, 0, 0};
  while (p < end) {
    uint64_t key, v;
    if (get_varint(&p, end, &key) || key > 0xFFFFFFFFull) goto bad;
    uint32_t wt = (uint32_t)(key & 7);
    uint64_t fn = key >> 3;
    if (fn == 0) goto bad;
    if (fn == 1) {
      if (wt == 2) { /* packed */
        uint64_t l;
        if (get_varint(&p, end, &l) || l > (uint64_t)(end - p)) goto bad;
        const uint8_t* lim = p + l;
        while (p < lim) {
          if (get_varint(&p, lim, &v)) goto bad;
          if (bvec_push(&bits, v != 0)) goto nomem;
        }
      } else if (wt == 0) { /* unpacked element */
        if (get_varint(&p, end, &v)) goto bad;
        if (bvec_push(&bits, v != 0)) goto nomem;
      } else {
        goto bad; /* wire-type mismatch on a known field */
      }
    } else if (skip_field(&p, end, wt, fn, 0)) {
      goto bad;
    }
  }
  out->m = bits.n;
  out->bits = bits.v;
  if (out->m == 0) {
    free(out->bits);
    out->bits = NULL;
  }
  return OB_OK;
bad:
  free(bits.v);
  return OB_EDECODE;
nomem:
  free(bits.v);
  return OB_ENOMEM;
}

/* ---- ZoneMap and the SsTable::get gate ---- */

int ob_bytes_cmp(const uint8_t* a, uint64_t alen, const uint8_t* b, uint64_t blen) {
  uint64_t n = alen < blen ? alen : blen;
  int c = n ? memcmp(a, b, (size_t)n) : 0;
  if (c) return c < 0 ? -1 : 1;
  return alen < blen ? -1 : (alen > blen ? 1 : 0);
}

void ob_zone_init(ob_zone* z) { memset(z, 0, sizeof(*z)); }

void ob_zone_free(ob_zone* z) {
  free(z->min);
  free(z->max);
  ob_zone_init(z);
}

static int copy_bytes(uint8_t** dst, uint64_t* dlen, const uint8_t* src, uint64_t len) {
  uint8_t* p = (uint8_t*)malloc(len ? (size_t)len : 1);
  if (!p) return OB_ENOMEM;
  if (len) memcpy(p, src, (size_t)len);
  free(*dst);
  *dst = p;
  *dlen = len;
  return OB_OK;
}

int ob_zone_set(ob_zone* z, const uint8_t* min, uint64_t min_len, int has_min, const uint8_t* max,
                uint64_t max_len, int has_max) {
  ob_zone_free(z);
  if (has_min && copy_bytes(&z->min, &z->min_len, min, min_len)) return OB_ENOMEM;
  if (has_max && copy_bytes(&z->max, &z->max_len, max, max_len)) return OB_ENOMEM;
  z->has_min = has_min;
  z->has_max = has_max;
  return OB_OK;
}

int ob_zone_update(ob_zone* z, const uint8_t* key, uint64_t len) {
  /* zonemap.rs:22-26: min = key if none or key < min */
  if (!z->has_min || ob_bytes_cmp(key, len, z->min, z->min_len) < 0) {
    if (copy_bytes(&z->min, &z->min_len, key, len)) return OB_ENOMEM;
    z->has_min = 1;
  }
  /* zonemap.rs:27-31: max = key if none or key > max */
  if (!z->has_max || ob_bytes_cmp(key, len, z->max, z->max_len) > 0) {
    if (copy_bytes(&z->max, &z->max_len, key, len)) return OB_ENOMEM;
    z->has_max = 1;
  }
  return OB_OK;
}

int ob_zone_contains(const ob_zone* z, const uint8_t* key, uint64_t len) {
  if (!z || !z->has_min || !z->has_max) return 1; /* zonemap.rs:40 */
  return ob_bytes_cmp(key, len, z->min, z->min_len) >= 0 &&
         ob_bytes_cmp(key, len, z->max, z->max_len) <= 0; /* zonemap.rs:39 */
}

int ob_probe_gated_var(const ob_filter* const* fs, const ob_zone* const* zones, uint32_t nf,
                       const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* hits) {
  uint64_t words = (n + 63) / 64;
  for (uint32_t f = 0; f < nf; ++f)
    if (n && fs[f]->m == 0) return OB_EZEROM;
  memset(hits, 0, (size_t)(words * nf * sizeof(uint64_t)));
  for (uint64_t k = 0; k < n; ++k) {
    const uint8_t* key = bytes + offsets[k];
    uint64_t len = offsets[k + 1] - offsets[k];
    for (uint32_t f = 0; f < nf; ++f) {
      /* src/sstable.rs:138: `!zone_map.contains(key) || !bloom.may_contain(key)` */
      if (ob_zone_contains(zones ? zones[f] : NULL, key, len) && ob_may_contain(fs[f], key, len) == 1)
        hits[(uint64_t)f * words + (k >> 6)] |= (uint64_t)1 << (k & 63);
    }
  }
  return OB_OK;
}

/* ---- TableMeta codec (src/sstable.rs:31-37,74-81,96-108) ---- */

int ob_utf8_valid(const uint8_t* p, uint64_t n) {
  /* Unicode 3.9 well-formed byte sequences (what Rust's from_utf8 accepts):
   * no overlongs, no surrogates D800-DFFF, nothing above U+10FFFF. */
  uint64_t i = 0;
  while (i < n) {
    uint8_t c = p[i];
    if (c < 0x80) {
      ++i;
      continue;
    }
    int len;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) len = 2;
    else if (c == 0xE0) { len = 3; lo = 0xA0; }
    else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) len = 3;
    else if (c == 0xED) { len = 3; hi = 0x9F; }
    else if (c == 0xF0) { len = 4; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) len = 4;
    else if (c == 0xF4) { len = 4; hi = 0x8F; }
    else return 0;
    if (n - i < (uint64_t)len) return 0;
    if (p[i + 1] < lo || p[i + 1] > hi) return 0;
    for (int k = 2; k < len; ++k)
      if (p[i + k] < 0x80 || p[i + k] > 0xBF) return 0;
    i += (uint64_t)len;
  }
  return 1;
}

static uint64_t str_field_len(uint64_t l) { return 1 + varint_len(l) + l; }

uint64_t ob_meta_encode(const ob_filter* bloom, const ob_zone* zone, uint8_t* out, uint64_t cap) {
  uint64_t bl = 0, zl = 0, total = 0;
  if (bloom) {
    bl = ob_encode(bloom, NULL, 0);
    total += 1 + varint_len(bl) + bl;
  }
  if (zone) {
    if (zone->has_min) zl += str_field_len(zone->min_len);
    if (zone->has_max) zl += str_field_len(zone->max_len);
    total += 1 + varint_len(zl) + zl;
  }
  if (!out || cap < total) return total;
  uint8_t* p = out;
  if (bloom) {
    *p++ = 0x0A; /* field 1 (bloom), length-delimited */
    p = put_varint(p, bl);
    p += ob_encode(bloom, p, bl);
  }
  if (zone) {
    *p++ = 0x12; /* field 2 (zone_map), length-delimited */
    p = put_varint(p, zl);
    if (zone->has_min) {
      *p++ = 0x0A;
      p = put_varint(p, zone->min_len);
      if (zone->min_len) memcpy(p, zone->min, (size_t)zone->min_len);
      p += zone->min_len;
    }
    if (zone->has_max) {
      *p++ = 0x12;
      p = put_varint(p, zone->max_len);
      if (zone->max_len) memcpy(p, zone->max, (size_t)zone->max_len);
      p += zone->max_len;
    }
  }
  return total;
}

void ob_meta_free(ob_meta* m) {
  ob_free(&m->bloom);
  ob_zone_free(&m->zone);
  m->has_bloom = m->has_zone = 0;
}

/* ZoneMapProto::merge: each present string replaces the current value. */
static int merge_zone(const uint8_t* p, const uint8_t* end, ob_zone* z) {
  while (p < end) {
    uint64_t key, l;
    if (get_varint(&p, end, &key) || key > 0xFFFFFFFFull) return OB_EDECODE;
    uint32_t wt = (uint32_t)(key & 7);
    uint64_t fn = key >> 3;
    if (fn == 0) return OB_EDECODE;
    if (fn == 1 || fn == 2) {
      if (wt != 2) return OB_EDECODE;
      if (get_varint(&p, end, &l) || l > (uint64_t)(end - p)) return OB_EDECODE;
      if (!ob_utf8_valid(p, l)) return OB_EDECODE;
      if (fn == 1) {
        if (copy_bytes(&z->min, &z->min_len, p, l)) return OB_ENOMEM;
        z->has_min = 1;
      } else {
        if (copy_bytes(&z->max, &z->max_len, p, l)) return OB_ENOMEM;
        z->has_max = 1;
      }
      p += l;
    } else if (skip_field(&p, end, wt, fn, 0)) {
      return OB_EDECODE;
    }
  }
  return OB_OK;
}

int ob_meta_decode(const uint8_t* in, uint64_t len, ob_meta* out) {
  const uint8_t* p = in;
  const uint8_t* end = in + len;
  int rc = OB_OK;
  memset(out, 0, sizeof(*out));
  while (p < end) {
    uint64_t key, l;
    if (get_varint(&p, end, &key) || key > 0xFFFFFFFFull) { rc = OB_EDECODE; break; }
    uint32_t wt = (uint32_t)(key & 7);
    uint64_t fn = key >> 3;
    if (fn == 0) { rc = OB_EDECODE; break; }
    if (fn == 1 || fn == 2) {
      if (wt != 2) { rc = OB_EDECODE; break; }
      if (get_varint(&p, end, &l) || l > (uint64_t)(end - p)) { rc = OB_EDECODE; break; }
      if (fn == 1) {
        /* BloomProto::merge: the repeated bits of this occurrence append */
        ob_filter part = {NULL, 0};
        if ((rc = ob_decode(p, l, &part))) break;
        if (part.m) {
          uint8_t* nb = (uint8_t*)realloc(out->bloom.bits, (size_t)(out->bloom.m + part.m));
          if (!nb) { ob_free(&part); rc = OB_ENOMEM; break; }
          memcpy(nb + out->bloom.m, part.bits, (size_t)part.m);
          out->bloom.bits = nb;
          out->bloom.m += part.m;
        }
        ob_free(&part);
        out->has_bloom = 1;
      } else {
        if ((rc = merge_zone(p, p + l, &out->zone))) break;
        out->has_zone = 1;
      }
      p += l;
    } else if (skip_field(&p, end, wt, fn, 0)) {
      rc = OB_EDECODE;
      break;
    }
  }
  if (rc) ob_meta_free(out);
  return rc;
}

/* ---- SSTable data file: split, binary search, base64, get ---- */

int ob_table_index(const uint8_t* data, uint64_t len, ob_table* t) {
  memset(t, 0, sizeof(*t));
  t->data = data;
  t->len = len;
  uint64_t cap = 0;
  uint64_t i = 0;
  while (i < len) {
    uint64_t j = i;
    while (j < len && data[j] != '\n') ++j;
    if (j > i) { /* .filter(|line| !line.is_empty()) */
      if (t->nlines == cap) {
        cap = cap ? 2 * cap : 64;
        uint64_t* ns = (uint64_t*)realloc(t->start, cap * 8);
        if (!ns) return OB_ENOMEM;
        t->start = ns;
        uint64_t* ne = (uint64_t*)realloc(t->end, cap * 8);
        if (!ne) return OB_ENOMEM;
        t->end = ne;
      }
      t->start[t->nlines] = i;
      t->end[t->nlines] = j;
      ++t->nlines;
    }
    i = j + 1;
  }
  return OB_OK;
}

void ob_table_free(ob_table* t) {
  free(t->start);
  free(t->end);
  memset(t, 0, sizeof(*t));
}

int64_t ob_table_search(const ob_table* t, const uint8_t* key, uint64_t klen, uint64_t* val,
                        uint64_t* val_len) {
  uint64_t lo = 0, hi = t->nlines;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    const uint8_t* line = t->data + t->start[mid];
    uint64_t ll = t->end[mid] - t->start[mid];
    const uint8_t* tab = (const uint8_t*)memchr(line, '\t', (size_t)ll);
    if (!tab) break; /* no SEP: `else { break; }` */
    uint64_t pos = (uint64_t)(tab - line);
    int c = ob_bytes_cmp(line, pos, key, klen);
    if (c < 0) lo = mid + 1;
    else if (c > 0) hi = mid;
    else {
      if (val) *val = t->start[mid] + pos + 1;
      if (val_len) *val_len = ll - pos - 1;
      return (int64_t)mid;
    }
  }
  return -1;
}

static int b64_sym(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

int64_t ob_b64_decode(const uint8_t* in, uint64_t len, uint8_t* out) {
  if (len % 4) return -1; /* canonical padding: whole quads only */
  uint64_t pad = 0;
  if (len && in[len - 1] == '=') pad = (len >= 2 && in[len - 2] == '=') ? 2 : 1;
  uint64_t o = 0;
  for (uint64_t q = 0; q < len; q += 4) {
    int last = q + 4 == len;
    int v[4];
    for (int k = 0; k < 4; ++k) {
      if (last && k >= 4 - (int)pad) {
        v[k] = 0; /* '=' only at the tail */
        continue;
      }
      v[k] = b64_sym(in[q + k]);
      if (v[k] < 0) return -1;
    }
    uint32_t w = (uint32_t)v[0] << 18 | (uint32_t)v[1] << 12 | (uint32_t)v[2] << 6 | (uint32_t)v[3];
    int nout = last ? 3 - (int)pad : 3;
    if (last && pad == 2 && (v[1] & 0x0F)) return -1; /* trailing bits must be zero */
    if (last && pad == 1 && (v[2] & 0x03)) return -1;
    if (out) {
      out[o] = (uint8_t)(w >> 16);
      if (nout > 1) out[o + 1] = (uint8_t)(w >> 8);
      if (nout > 2) out[o + 2] = (uint8_t)w;
    }
    o += (uint64_t)nout;
  }
  return (int64_t)o;
}

uint64_t ob_b64_encode(const uint8_t* in, uint64_t len, uint8_t* out) {
  static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  uint64_t o = 0;
  for (uint64_t i = 0; i < len; i += 3) {
    uint64_t r = len - i;
    uint32_t w = (uint32_t)in[i] << 16 | (r > 1 ? (uint32_t)in[i + 1] << 8 : 0) | (r > 2 ? in[i + 2] : 0);
    if (out) {
      out[o] = (uint8_t)A[w >> 18];
      out[o + 1] = (uint8_t)A[(w >> 12) & 63];
      out[o + 2] = r > 1 ? (uint8_t)A[(w >> 6) & 63] : '=';
      out[o + 3] = r > 2 ? (uint8_t)A[w & 63] : '=';
    }
    o += 4;
  }
  return o;
}

int ob_get_many(const ob_table* const* tables, uint32_t nt, const uint64_t* hits,
                const uint8_t* bytes, const uint64_t* offsets, uint64_t n, int32_t* which,
                uint64_t* val_off, uint8_t* vals, uint64_t cap, uint64_t* total) {
  uint64_t words = (n + 63) / 64, acc = 0;
  int64_t* got_line = (int64_t*)malloc((n ? n : 1) * 8);
  uint64_t* vstart = (uint64_t*)malloc((n ? n : 1) * 8);
  uint64_t* vlen = (uint64_t*)malloc((n ? n : 1) * 8);
  if (!got_line || !vstart || !vlen) {
    free(got_line);
    free(vstart);
    free(vlen);
    return OB_ENOMEM;
  }
  for (uint64_t k = 0; k < n; ++k) {
    const uint8_t* key = bytes + offsets[k];
    uint64_t klen = offsets[k + 1] - offsets[k];
    which[k] = -1;
    val_off[k] = acc;
    for (uint32_t t = 0; t < nt; ++t) { /* tables.iter().rev(): newest first */
      if (hits && !((hits[(uint64_t)t * words + (k >> 6)] >> (k & 63)) & 1)) continue;
      uint64_t vs, vl;
      if (ob_table_search(tables[t], key, klen, &vs, &vl) < 0) continue; /* Ok(None) */
      int64_t d = ob_b64_decode(tables[t]->data + vs, vl, NULL);
      if (d < 0) continue; /* Err(..): `if let Ok(Some(v))` skips it */
      which[k] = (int32_t)t;
      vstart[k] = vs;
      vlen[k] = vl;
      acc += (uint64_t)d;
      break;
    }
  }
  val_off[n] = acc;
  *total = acc;
  if (vals && cap >= acc)
    for (uint64_t k = 0; k < n; ++k)
      if (which[k] >= 0) ob_b64_decode(tables[which[k]]->data + vstart[k], vlen[k], vals + val_off[k]);
  free(got_line);
  free(vstart);
  free(vlen);
  return OB_OK;
}

/* ---- SsTable::create (src/sstable.rs:56-72) ---- */

static const uint8_t* g_sort_kb;
static const uint64_t* g_sort_ko;

static int entry_cmp(const void* x, const void* y) {
  uint64_t i = *(const uint64_t*)x, j = *(const uint64_t*)y;
  int c = ob_bytes_cmp(g_sort_kb + g_sort_ko[i], g_sort_ko[i + 1] - g_sort_ko[i], g_sort_kb + g_sort_ko[j],
                       g_sort_ko[j + 1] - g_sort_ko[j]);
  if (c) return c;
  return i < j ? -1 : (i > j); /* Rust's sort_by is stable: equal keys keep input order */
}

uint64_t ob_sstable_create(const uint8_t* kbytes, const uint64_t* koff, const uint8_t* vbytes,
                           const uint64_t* voff, uint64_t n, uint8_t* out, uint64_t cap) {
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i)
    total += (koff[i + 1] - koff[i]) + 1 + 4 * ((voff[i + 1] - voff[i] + 2) / 3) + 1;
  if (!out || cap < total || !n) return total;
  uint64_t* ord = (uint64_t*)malloc(n * 8);
  if (!ord) return 0;
  for (uint64_t i = 0; i < n; ++i) ord[i] = i;
  g_sort_kb = kbytes;
  g_sort_ko = koff;
  qsort(ord, (size_t)n, 8, entry_cmp); /* not thread-safe: test infrastructure only */
  uint8_t* p = out;
  for (uint64_t r = 0; r < n; ++r) {
    uint64_t i = ord[r];
    uint64_t kl = koff[i + 1] - koff[i];
    memcpy(p, kbytes + koff[i], (size_t)kl);
    p += kl;
    *p++ = '\t';                                                           /* SEP */
    p += ob_b64_encode(vbytes + voff[i], voff[i + 1] - voff[i], p);        /* STANDARD.encode */
    *p++ = '\n';                                                           /* NL */
  }
  free(ord);
  return total;
}

/* ---- synthetic workload ---- */

uint64_t ob_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void ob_gen_keys(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out) {
  static const char hex[] = "0123456789abcdef";
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t v = ob_splitmix64((seed << 32) + first + i);
    uint8_t* o = out + i * 16;
    for (int d = 0; d < 16; ++d) o[d] = (uint8_t)hex[(v >> (60 - 4 * d)) & 15];
  }
}

int ob_table_rebuild(const ob_table* t, uint64_t m, ob_filter* bloom, ob_zone* zone, uint64_t* bad_line) {
  /* src/sstable.rs:110-120 */
  int rc = ob_new(bloom, m); /* BloomFilter::new(1024) in the reference; m here */
  if (rc) return rc;
  ob_zone_init(zone);
  if (bad_line) *bad_line = UINT64_MAX;
  for (uint64_t l = 0; l < t->nlines; ++l) {
    const uint8_t* line = t->data + t->start[l];
    const uint64_t n = t->end[l] - t->start[l];
    const uint8_t* tab = memchr(line, '\t', n);
    if (!tab) continue; /* `if let Some(pos)`: lines without SEP are skipped */
    const uint64_t kl = (uint64_t)(tab - line);
    if (!ob_utf8_valid(line, kl)) { /* from_utf8(..).map_err(..)? */
      if (bad_line) *bad_line = l;
      return OB_EUTF8;
    }
    if ((rc = ob_insert(bloom, line, kl))) return rc;
    if ((rc = ob_zone_update(zone, line, kl))) return rc;
  }
  return OB_OK;
}
