/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see zd_oracle.h).
 *
 * Plain-C restatement of the reference Rust decoder
 * AchilleBailly/zstd-decompressor (zstd-decompressor/src/…).  Every function
 * cites the reference item it follows.  Reference quirks are kept on purpose
 * (SURVEY.md §2.1): D1 nbSeq+0x7F, D2 nbSeq==0 fails, D3 power-of-two weight
 * totals panic, D4 no window trimming, D5 checksum ignored, D7 dict id
 * ignored, D8 regenerated size ignored / u16 stream sizes, D9 zero offset
 * panics.  Where the reference (built in debug, as `cargo run/test` does)
 * would panic or never terminate, this returns ZD_E_REF_PANIC.
 *
 * Parity: pinned by the reference's KATs (tests/golden/kat.json) and by
 * libzstd goldens on in-domain frames; the reference itself is not buildable
 * here (no cargo/rustc, crates not vendored).
 */
#include "zd_oracle.h"
#include "../include/zd.h"

#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

#define TRY(x) do { int _r = (x); if (_r) return _r; } while (0)

static int fail(zdo_err* e, int code, int64_t a, int64_t b) {
  if (e) { e->code = code; e->a = a; e->b = b; }
  return code;
}

/* (X >> lo) & mask(len) where X is d[0..n) read as a little-endian integer;
 * len <= 64 and [lo, lo+len) inside the data. */
static uint64_t le_bits(const uint8_t* d, size_t n, uint64_t lo, unsigned len) {
  if (len == 0) return 0;
  size_t b0 = (size_t)(lo >> 3), b1 = (size_t)((lo + len - 1) >> 3);
  u128 acc = 0;
  for (size_t i = b1 + 1; i-- > b0;) acc = (acc << 8) | d[i];
  (void)n;
  acc >>= (lo & 7);
  return (uint64_t)(len == 64 ? acc : (acc & ((((u128)1) << len) - 1)));
}

/* ---------------- parsing.rs ---------------- */

/* ForwardByteParser (parsing.rs:9-112) */
typedef struct { const uint8_t* p; size_t n; } fbp;

static int fbp_u8(fbp* b, uint8_t* v, zdo_err* e) {            /* parsing.rs:39-50 */
  if (!b->n) return fail(e, ZD_E_NOT_ENOUGH_BYTES, 1, 0);
  *v = *b->p++; b->n--; return 0;
}
static int fbp_slice(fbp* b, size_t len, const uint8_t** s, zdo_err* e) { /* parsing.rs:63-79 */
  if (len == 0) return fail(e, ZD_E_EMPTY_SLICE, 0, 0);
  if (b->n < len) return fail(e, ZD_E_NOT_ENOUGH_BYTES, (int64_t)len, (int64_t)b->n);
  *s = b->p; b->p += len; b->n -= len; return 0;
}
static int fbp_le_u32(fbp* b, uint32_t* v, zdo_err* e) {        /* parsing.rs:82-95 */
  if (b->n < 4) return fail(e, ZD_E_NOT_ENOUGH_BYTES, 4, (int64_t)b->n);
  *v = (uint32_t)b->p[0] | ((uint32_t)b->p[1] << 8) | ((uint32_t)b->p[2] << 16) | ((uint32_t)b->p[3] << 24);
  b->p += 4; b->n -= 4; return 0;
}
static int fbp_le_u16(fbp* b, uint16_t* v, zdo_err* e) {        /* parsing.rs:98-111 */
  if (b->n < 2) return fail(e, ZD_E_NOT_ENOUGH_BYTES, 2, (int64_t)b->n);
  *v = (uint16_t)(b->p[0] | (b->p[1] << 8));
  b->p += 2; b->n -= 2; return 0;
}

/* ForwardBitParser (parsing.rs:114-189): LSB-first (bitbuffer LittleEndian). */
typedef struct { const uint8_t* d; size_t nbytes; uint64_t readable, pos; } fwbits;

static int fw_new(fwbits* f, const uint8_t* d, size_t n, zdo_err* e) { /* parsing.rs:131-140 */
  if (n == 0) return fail(e, ZD_E_EMPTY_INPUT_DATA, 0, 0);
  f->d = d; f->nbytes = n; f->readable = (uint64_t)n * 8; f->pos = 0; return 0;
}
static uint64_t fw_bytes_read(const fwbits* f) {                   /* parsing.rs:122-126 */
  return f->pos / 8 + (f->pos % 8 > 0);
}
static int fw_take(fwbits* f, uint64_t len, uint64_t* v, zdo_err* e) { /* parsing.rs:152-170 */
  if (f->nbytes * 8 - f->pos < len) return fail(e, ZD_E_NOT_ENOUGH_BITS, (int64_t)len, (int64_t)f->readable);
  if (len > 64) return fail(e, ZD_E_MAX_READABLE_BITS_EXCEEDED, (int64_t)len, 0);
  *v = le_bits(f->d, f->nbytes, f->pos, (unsigned)len);
  f->readable -= len; f->pos += len; return 0;
}
static int fw_peek(const fwbits* f, uint64_t len, uint64_t* v, zdo_err* e) { /* parsing.rs:173-188 */
  if (f->nbytes * 8 - f->pos < len) return fail(e, ZD_E_NOT_ENOUGH_BITS, (int64_t)len, (int64_t)(f->nbytes * 8));
  if (len > 64) return fail(e, ZD_E_MAX_READABLE_BITS_EXCEEDED, (int64_t)len, 0);
  *v = le_bits(f->d, f->nbytes, f->pos, (unsigned)len); return 0;
}

/* BackwardBitParser (parsing.rs:191-259).  The reference reverses the bytes
 * and reads BigEndian from bit `pos`; reading k bits at pos of the reversed
 * stream equals bits [8n-pos-k, 8n-pos) of the original little-endian
 * integer, which is what we extract (no copy). */
typedef struct { const uint8_t* d; size_t nbytes; uint64_t readable, pos; } bwbits;

static int bw_new(bwbits* b, const uint8_t* d, size_t n, zdo_err* e) { /* parsing.rs:200-220 */
  if (n == 0) return fail(e, ZD_E_EMPTY_INPUT_DATA, 0, 0);
  if (d[n - 1] == 0) return fail(e, ZD_E_NULL_BYTE, 0, 0);
  unsigned i = 1;
  while ((d[n - 1] & (1u << (8 - i))) == 0) i++;
  b->d = d; b->nbytes = n; b->readable = (uint64_t)n * 8 - i; b->pos = i; return 0;
}
static int bw_take(bwbits* b, uint64_t len, uint64_t* v, zdo_err* e) { /* parsing.rs:228-254 */
  if (b->nbytes * 8 - b->pos < len) return fail(e, ZD_E_NOT_ENOUGH_BITS, (int64_t)len, (int64_t)b->readable);
  if (len > 64) return fail(e, ZD_E_MAX_READABLE_BITS_EXCEEDED, (int64_t)len, 0);
  if (len == 0) { *v = 0; return 0; }
  *v = le_bits(b->d, b->nbytes, b->nbytes * 8 - b->pos - len, (unsigned)len);
  b->readable -= len; b->pos += len; return 0;
}

/* ---------------- utils.rs ---------------- */
static int discrete_log2_u64(uint64_t v, unsigned* out) {   /* utils.rs:33-40 (asserts v > 0) */
  if (v == 0) return ZD_E_REF_PANIC;
  unsigned r = 0; while (v >>= 1) r++;
  *out = r; return 0;
}

/* ---------------- decoders/fse.rs ---------------- */
#define MAX_AL 9            /* fse.rs:13 */
#define MAX_SYMBOL 256      /* fse.rs:14 */

typedef struct { uint16_t output, baseline, bits; } fse_state;  /* fse.rs:72-76 */
typedef struct { fse_state t[1 << MAX_AL]; uint8_t al; } fse_table;  /* fse.rs:86-89 */

/* parse_fse_table (fse.rs:16-69). dist has room for MAX_SYMBOL entries;
 * zeros pushed beyond that are only counted (the reference then fails). */
static int parse_fse_table(fwbits* in, uint8_t* al_out, int16_t* dist, size_t* nsym_out, zdo_err* e) {
  uint64_t v;
  TRY(fw_take(in, 4, &v, e));
  unsigned al = (unsigned)v + 5;
  if (al > MAX_AL) return fail(e, ZD_E_LARGE_ACCURACY_LOG, al, 0);
  int32_t remaining = 1 << al;
  size_t n_sym = 0;
  while (remaining > 0 && n_sym < MAX_SYMBOL) {
    unsigned lg; discrete_log2_u64((uint64_t)remaining + 1, &lg);
    unsigned bits_to_read = lg + 1;
    uint64_t pk; TRY(fw_peek(in, bits_to_read, &pk, e));
    uint16_t peeked = (uint16_t)pk;
    uint16_t lower_mask = (uint16_t)((1u << (bits_to_read - 1)) - 1);
    uint16_t threshold = (uint16_t)((1u << bits_to_read) - 1 - ((uint16_t)remaining + 1));
    int16_t decoded;
    if ((uint16_t)(peeked & lower_mask) < threshold) {
      TRY(fw_take(in, bits_to_read - 1, &v, e)); decoded = (int16_t)v;
    } else if (peeked > lower_mask) {
      TRY(fw_take(in, bits_to_read, &v, e)); decoded = (int16_t)((int16_t)v - (int16_t)threshold);
    } else {
      TRY(fw_take(in, bits_to_read, &v, e)); decoded = (int16_t)v;
    }
    int16_t proba = (int16_t)(decoded - 1);
    remaining -= proba < 0 ? -proba : proba;
    if (n_sym < MAX_SYMBOL) dist[n_sym] = proba;
    n_sym++;
    if (proba == 0) {
      for (;;) {
        TRY(fw_take(in, 2, &v, e));
        for (uint64_t z = 0; z < v; z++) { if (n_sym < MAX_SYMBOL) dist[n_sym] = 0; n_sym++; }
        if (v != 3) break;
      }
    }
  }
  if (remaining != 0 || n_sym >= MAX_SYMBOL) return fail(e, ZD_E_CORRUPTED_TABLE, 0, 0);
  *al_out = (uint8_t)al; *nsym_out = n_sym; return 0;
}

static unsigned ceil_log2(size_t n) {  /* f32::log2(n).ceil() as u32, exact for n <= 512; 0 -> 0 (saturating cast of -inf) */
  unsigned r = 0; while (((size_t)1 << r) < n) r++; return r;
}

/* FseTable::from_distribution (fse.rs:110-202) */
static int fse_from_distribution(uint8_t al, const int16_t* dist, size_t n, fse_table* out, zdo_err* e) {
  if (al > MAX_AL) return fail(e, ZD_E_LARGE_ACCURACY_LOG, al, 0);
  size_t T = (size_t)1 << al;
  uint8_t filled[1 << MAX_AL], has_bl[1 << MAX_AL];
  memset(filled, 0, T); memset(has_bl, 0, T);
  size_t zero_pos = T;
  for (size_t s = 0; s < n; s++) {                       /* fse.rs:121-133 */
    if (dist[s] == -1) {
      if (zero_pos == 0) return ZD_E_REF_PANIC;          /* usize underflow */
      zero_pos--;
      out->t[zero_pos].output = (uint16_t)s; out->t[zero_pos].baseline = 0; out->t[zero_pos].bits = al;
      filled[zero_pos] = 1; has_bl[zero_pos] = 1;
    }
  }
  size_t position = 0, step = (T >> 1) + (T >> 3) + 3, mask = T - 1;   /* fse.rs:136-157 */
  for (size_t s = 0; s < n; s++) {
    for (int16_t k = 0; k < dist[s]; k++) {
      out->t[position].output = (uint16_t)s; filled[position] = 1; has_bl[position] = 0;
      position = (position + step) & mask;
      size_t guard = 0;
      while (position >= zero_pos) {
        position = (position + step) & mask;
        if (++guard > T) return ZD_E_REF_PANIC;          /* reference loops forever */
      }
    }
  }
  for (size_t i = 0; i < T; i++) if (!filled[i]) return fail(e, ZD_E_CORRUPTED_TABLE, 0, 0); /* fse.rs:160-166 */
  for (size_t sym = 0; sym < n; sym++) {                  /* fse.rs:169-189 */
    size_t grouped[1 << MAX_AL], num_states = 0;
    for (size_t i = 0; i < T; i++) if (out->t[i].output == (uint16_t)sym) grouped[num_states++] = i;
    size_t parts = (size_t)1 << ceil_log2(num_states);
    size_t base_width = T / parts;
    unsigned base_nb; if (discrete_log2_u64(base_width, &base_nb)) return ZD_E_REF_PANIC;
    uint16_t baseline = 0;
    for (size_t i = parts - num_states; i < parts; i++) {
      size_t new_i = i % num_states;
      unsigned add = new_i != i ? 1 : 0, mult = new_i != i ? 2 : 1;
      out->t[grouped[new_i]].bits = (uint16_t)(base_nb + add);
      out->t[grouped[new_i]].baseline = baseline;
      has_bl[grouped[new_i]] = 1;
      baseline = (uint16_t)(baseline + (uint16_t)base_width * mult);
    }
  }
  for (size_t i = 0; i < T; i++) if (!has_bl[i]) return ZD_E_REF_PANIC;  /* .unwrap() on None (fse.rs:193-197) */
  out->al = al;
  return 0;
}

/* FseDecoder (fse.rs:230-323) / RLEDecoder (rle.rs:6-34) behind one struct. */
typedef struct {
  const fse_table* table;  /* NULL for RLE */
  uint16_t rle;
  size_t cur;
  int has_next; uint16_t next;
} bitdec;

static int dec_initialize(bitdec* d, bwbits* bs, zdo_err* e) {   /* fse.rs:280-288 */
  if (!d->table) return 0;                                       /* rle.rs:15-17 */
  uint64_t v; TRY(bw_take(bs, d->table->al, &v, e));
  d->next = d->table->t[v].output; d->has_next = 1; d->cur = (size_t)v; return 0;
}
static uint64_t dec_expected_bits(const bitdec* d) {              /* fse.rs:290-292 */
  return d->table ? d->table->t[d->cur].bits : 0;
}
static int dec_symbol(bitdec* d, uint16_t* s) {                   /* fse.rs:294-303 */
  if (!d->table) { *s = d->rle; return 0; }
  if (!d->has_next) return ZD_E_REF_PANIC;
  *s = d->next; d->has_next = 0; return 0;
}
static int dec_update(bitdec* d, bwbits* bs, zdo_err* e) {        /* fse.rs:305-318 */
  if (!d->table) return 0;
  if (d->has_next) return ZD_E_REF_PANIC;
  uint64_t v; TRY(bw_take(bs, dec_expected_bits(d), &v, e));
  size_t ns = (size_t)v + d->table->t[d->cur].baseline;
  if (ns >= ((size_t)1 << d->table->al)) return ZD_E_REF_PANIC;   /* index out of bounds */
  d->next = d->table->t[ns].output; d->has_next = 1; d->cur = ns; return 0;
}

/* AlternatingDecoder (alternating.rs:8-69) */
typedef struct { bitdec a, b; int last_updated_is_first, last_read_is_first; } altdec;

static int alt_initialize(altdec* d, bwbits* bs, zdo_err* e) {
  TRY(dec_initialize(&d->a, bs, e)); TRY(dec_initialize(&d->b, bs, e));
  d->last_updated_is_first = 0; d->last_read_is_first = 0; return 0;
}
static uint64_t alt_expected(const altdec* d) {
  return d->last_updated_is_first ? dec_expected_bits(&d->b) : dec_expected_bits(&d->a);
}
static int alt_symbol(altdec* d, uint16_t* s) {
  if (d->last_read_is_first) { d->last_read_is_first = 0; return dec_symbol(&d->b, s); }
  d->last_read_is_first = 1; return dec_symbol(&d->a, s);
}
static int alt_update(altdec* d, bwbits* bs, zdo_err* e) {
  if (d->last_updated_is_first) { d->last_updated_is_first = 0; return dec_update(&d->b, bs, e); }
  d->last_updated_is_first = 1; return dec_update(&d->a, bs, e);
}

/* ---------------- decoders/huffman.rs ---------------- */
enum { H_ABSENT = 0, H_SYMBOL = 1, H_TREE = 2 };
typedef struct { uint8_t kind, payload; int32_t left, right; } hnode;
typedef struct { hnode* n; size_t len, cap; } htree;   /* node 0 = root */

static int32_t h_alloc(htree* t) {
  if (t->len == t->cap) {
    size_t nc = t->cap ? t->cap * 2 : 64;
    hnode* nn = (hnode*)realloc(t->n, nc * sizeof(hnode));
    if (!nn) return -1;
    t->n = nn; t->cap = nc;
  }
  t->n[t->len].kind = H_ABSENT; t->n[t->len].payload = 0; t->n[t->len].left = t->n[t->len].right = -1;
  return (int32_t)t->len++;
}
static void h_free(htree* t) { free(t->n); t->n = NULL; t->len = t->cap = 0; }

/* HuffmanDecoder::insert (huffman.rs:132-159). returns 1 inserted, 0 not, <0 panic/oom */
static int h_insert(htree* t, int32_t node, uint8_t symbol, unsigned width) {
  if (width == 0) {
    if (t->n[node].kind == H_ABSENT) { t->n[node].kind = H_SYMBOL; t->n[node].payload = symbol; return 1; }
    return 0;
  }
  switch (t->n[node].kind) {
    case H_TREE: {
      int r = h_insert(t, t->n[node].left, symbol, width - 1);
      if (r) return r;
      return h_insert(t, t->n[node].right, symbol, width - 1);
    }
    case H_ABSENT: {
      int32_t l = h_alloc(t); if (l < 0) return ZD_E_NO_MEMORY;
      int32_t r = h_alloc(t); if (r < 0) return ZD_E_NO_MEMORY;
      t->n[node].kind = H_TREE; t->n[node].left = l; t->n[node].right = r;
      return h_insert(t, node, symbol, width);
    }
    default: return ZD_E_REF_PANIC;   /* "Trying to inster a symbol into another" */
  }
}

typedef struct { uint8_t sym, width; } symw;
static int symw_cmp(const void* x, const void* y) {  /* order after sort+reverse: width desc, symbol asc */
  const symw* a = (const symw*)x; const symw* b = (const symw*)y;
  if (a->width != b->width) return a->width > b->width ? -1 : 1;
  return (int)a->sym - (int)b->sym;
}

/* HuffmanDecoder::from_number_of_bits (huffman.rs:161-175) */
static int h_from_number_of_bits(const uint8_t* widths, size_t n, htree* t) {
  symw* s = (symw*)malloc((n ? n : 1) * sizeof(symw));
  if (!s) return ZD_E_NO_MEMORY;
  size_t k = 0;
  for (size_t i = 0; i < n; i++) if (widths[i]) { s[k].sym = (uint8_t)i; s[k].width = widths[i]; k++; }
  qsort(s, k, sizeof(symw), symw_cmp);
  t->len = 0;
  if (h_alloc(t) < 0) { free(s); return ZD_E_NO_MEMORY; }
  for (size_t i = 0; i < k; i++) {
    int r = h_insert(t, 0, s[i].sym, s[i].width);
    if (r < 0) { free(s); return r; }
  }
  free(s); return 0;
}

/* HuffmanDecoder::from_weights (huffman.rs:177-203): widths (0 = absent)
 * for weights.len()+1 symbols. */
static int h_widths_from_weights(const uint8_t* w, size_t nw, uint8_t* widths) {
  uint32_t sum = 0;
  for (size_t i = 0; i < nw; i++) {
    if (w[i]) {
      if (w[i] - 1 >= 32) return ZD_E_REF_PANIC;                     /* shift overflow */
      uint32_t add = 1u << (w[i] - 1);
      if (sum > UINT32_MAX - add) return ZD_E_REF_PANIC;             /* add overflow */
      sum += add;
    }
  }
  unsigned p; if (discrete_log2_u64(sum, &p)) return ZD_E_REF_PANIC;
  if (((uint64_t)1 << p) < sum) p += 1;
  if (p >= 32) return ZD_E_REF_PANIC;                                 /* 1u32 << 32 */
  uint8_t rest = (uint8_t)((1u << p) - sum);
  unsigned lm; if (discrete_log2_u64(rest, &lm)) return ZD_E_REF_PANIC;   /* D3 */
  unsigned manquant = lm + 1;
  for (size_t i = 0; i < nw; i++) {
    if (w[i]) {
      if (w[i] > p + 1) return ZD_E_REF_PANIC;                        /* u8 underflow */
      widths[i] = (uint8_t)(p + 1 - w[i]);
    } else widths[i] = 0;
  }
  if (manquant > p + 1) return ZD_E_REF_PANIC;
  widths[nw] = (uint8_t)(p + 1 - manquant);
  return 0;
}

static int h_from_weights(const uint8_t* w, size_t nw, htree* t) {
  uint8_t* widths = (uint8_t*)malloc(nw + 1);
  if (!widths) return ZD_E_NO_MEMORY;
  int r = h_widths_from_weights(w, nw, widths);
  if (!r) r = h_from_number_of_bits(widths, nw + 1, t);
  free(widths); return r;
}

/* HuffmanDecoder::decode (huffman.rs:205-218) */
static int h_decode(const htree* t, bwbits* bs, uint8_t* out, zdo_err* e) {
  int32_t node = 0;
  for (;;) {
    const hnode* h = &t->n[node];
    if (h->kind == H_SYMBOL) { *out = h->payload; return 0; }
    if (h->kind == H_ABSENT) return ZD_E_REF_PANIC;
    uint64_t bit; TRY(bw_take(bs, 1, &bit, e));
    node = bit ? h->right : h->left;
  }
}

/* HuffmanDecoder::parse_direct (huffman.rs:92-106) */
static int h_parse_direct(fbp* in, size_t num_weights, uint8_t** w, size_t* nw, zdo_err* e) {
  const uint8_t* data;
  TRY(fbp_slice(in, num_weights / 2 + num_weights % 2, &data, e));
  size_t nb = num_weights / 2 + num_weights % 2;
  uint8_t* res = (uint8_t*)malloc(2 * nb);
  if (!res) return ZD_E_NO_MEMORY;
  for (size_t i = 0; i < nb; i++) { res[2 * i] = data[i] >> 4; res[2 * i + 1] = data[i] & 15; }
  *w = res; *nw = num_weights; return 0;
}

/* HuffmanDecoder::parse_fse (huffman.rs:108-130) */
static int h_parse_fse(fbp* in, uint8_t compressed_size, uint8_t** w, size_t* nw, zdo_err* e) {
  const uint8_t* data;
  TRY(fbp_slice(in, compressed_size, &data, e));
  fwbits fw; fw_new(&fw, data, compressed_size, NULL);
  int16_t dist[MAX_SYMBOL]; size_t nsym; uint8_t al;
  TRY(parse_fse_table(&fw, &al, dist, &nsym, e));
  fse_table* tab = (fse_table*)malloc(sizeof(fse_table));
  if (!tab) return ZD_E_NO_MEMORY;
  int r = fse_from_distribution(al, dist, nsym, tab, e);
  if (r) { free(tab); return r; }
  bwbits bs;
  size_t br = (size_t)fw_bytes_read(&fw);
  r = bw_new(&bs, data + br, compressed_size - br, e);
  if (r) { free(tab); return r; }
  altdec d; memset(&d, 0, sizeof d); d.a.table = tab; d.b.table = tab;
  r = alt_initialize(&d, &bs, e);
  if (r) { free(tab); return r; }
  size_t cap = 64, len = 0;
  uint8_t* res = (uint8_t*)malloc(cap);
  /* the loop may not terminate in the reference when every remaining state
   * reads 0 bits (huffman.rs:121-124); bound it */
  uint64_t guard = 0, guard_max = (8 * (uint64_t)compressed_size + 2) * ((1u << al) + 2) * 2;
  while (res && alt_expected(&d) <= bs.readable) {
    if (++guard > guard_max) { free(res); free(tab); return ZD_E_REF_PANIC; }
    uint16_t s; r = alt_symbol(&d, &s);
    if (!r) {
      if (len == cap) { cap *= 2; uint8_t* nr = (uint8_t*)realloc(res, cap); if (!nr) { free(res); res = NULL; break; } res = nr; }
      res[len++] = (uint8_t)s;
      r = alt_update(&d, &bs, e);
    }
    if (r) { free(res); free(tab); return r; }
  }
  if (!res) { free(tab); return ZD_E_NO_MEMORY; }
  for (int k = 0; k < 2; k++) {
    uint16_t s; r = alt_symbol(&d, &s);
    if (r) { free(res); free(tab); return r; }
    if (len == cap) { cap *= 2; uint8_t* nr = (uint8_t*)realloc(res, cap); if (!nr) { free(res); free(tab); return ZD_E_NO_MEMORY; } res = nr; }
    res[len++] = (uint8_t)s;
  }
  free(tab);
  *w = res; *nw = len; return 0;
}

/* HuffmanDecoder::parse (huffman.rs:80-90) -> weights */
static int h_parse_weights(fbp* in, uint8_t** w, size_t* nw, zdo_err* e) {
  uint8_t header; TRY(fbp_u8(in, &header, e));
  if (header < 128) return h_parse_fse(in, header, w, nw, e);
  return h_parse_direct(in, (size_t)header - 127, w, nw, e);
}

static int h_parse(fbp* in, htree* t, zdo_err* e) {
  uint8_t* w = NULL; size_t nw = 0;
  TRY(h_parse_weights(in, &w, &nw, e));
  int r = h_from_weights(w, nw, t);
  free(w); return r;
}

/* ---------------- literals.rs ---------------- */
enum { LIT_RAW = 0, LIT_RLE = 1, LIT_COMPRESSED = 2, LIT_TREELESS = 3 };

typedef struct {
  int type;
  const uint8_t* data; size_t data_len;   /* raw data / compressed streams */
  uint8_t byte; uint32_t repeat;          /* RLE */
  int has_tree; htree tree;               /* Compressed */
  uint16_t jump[4];
} literals_section;

/* LiteralsSection::parse_header (literals.rs:135-206) */
static int lit_parse_header(fbp* in, int* type, size_t* regen, size_t* csize, int* nstreams, zdo_err* e) {
  uint8_t h; TRY(fbp_u8(in, &h, e));
  int lt = h & 3, sf = (h >> 2) & 3;
  if (lt == LIT_RAW || lt == LIT_RLE) {
    uint8_t b1, b2;
    switch (sf) {
      case 0: case 2: *regen = h >> 3; break;
      case 1: TRY(fbp_u8(in, &b1, e)); *regen = (size_t)(h >> 4) + ((size_t)b1 << 4); break;
      default:
        TRY(fbp_u8(in, &b1, e)); TRY(fbp_u8(in, &b2, e));
        *regen = (size_t)(h >> 4) + ((size_t)b1 << 4) + ((size_t)b2 << 12); break;
    }
    *csize = 0; *nstreams = 1;
  } else {
    const uint8_t* s;
    switch (sf) {
      case 0: case 1: {
        TRY(fbp_slice(in, 2, &s, e));
        uint32_t x = s[0] | (s[1] << 8);
        *regen = (size_t)(h >> 4) + ((size_t)(x & 0x3F) << 4); *csize = x >> 6; *nstreams = sf == 0 ? 1 : 4; break;
      }
      case 2: {
        TRY(fbp_slice(in, 3, &s, e));
        uint32_t x = s[0] | (s[1] << 8) | ((uint32_t)s[2] << 16);
        *regen = (size_t)(h >> 4) + ((size_t)(x & 0x3FF) << 4); *csize = (x >> 10) & 0x3FFF; *nstreams = 4; break;
      }
      default: {
        TRY(fbp_slice(in, 4, &s, e));
        uint32_t x = s[0] | (s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
        *regen = (size_t)(h >> 4) + ((size_t)(x & 0x3FFF) << 4); *csize = (x >> 14) & 0x3FFFF; *nstreams = 4; break;
      }
    }
  }
  *type = lt; return 0;
}

/* LiteralsSection::parse (literals.rs:88-133) */
static int lit_parse(fbp* in, literals_section* L, zdo_err* e) {
  size_t regen, csize; int nstreams, lt;
  memset(L, 0, sizeof *L);
  TRY(lit_parse_header(in, &lt, &regen, &csize, &nstreams, e));
  L->type = lt;
  if (lt == LIT_RAW) { TRY(fbp_slice(in, regen, &L->data, e)); L->data_len = regen; return 0; }
  if (lt == LIT_RLE) { TRY(fbp_u8(in, &L->byte, e)); L->repeat = (uint32_t)regen; return 0; }
  const uint8_t* cs; TRY(fbp_slice(in, csize, &cs, e));
  fbp ni = { cs, csize };
  if (lt == LIT_COMPRESSED) { L->has_tree = 1; TRY(h_parse(&ni, &L->tree, e)); }
  size_t total = ni.n;
  if (nstreams == 4) {
    uint16_t s1, s2, s3;
    TRY(fbp_le_u16(&ni, &s1, e)); TRY(fbp_le_u16(&ni, &s2, e)); TRY(fbp_le_u16(&ni, &s3, e));
    if ((size_t)s1 + s2 + s3 > total - 6) return fail(e, ZD_E_CORRUPTED_STREAMS_SIZE, 0, 0);
    size_t s4 = total - 6 - s1 - s2 - s3;
    L->jump[0] = s1; L->jump[1] = s2; L->jump[2] = s3; L->jump[3] = (uint16_t)s4;
  } else {
    L->jump[0] = (uint16_t)ni.n; L->jump[1] = L->jump[2] = L->jump[3] = 0;
  }
  L->data_len = ni.n;
  TRY(fbp_slice(&ni, ni.n, &L->data, e));
  return 0;
}

/* ---------------- decoding_context.rs ---------------- */
enum { M_PREDEFINED = 0, M_RLE = 1, M_FSE = 2, M_REPEAT = 3 };
typedef struct { int mode; uint8_t rle; fse_table* table; } sym_mode;   /* SymbolCompressionMode (sequences.rs:256-261) */

typedef struct {
  int has_huffman; htree huffman;                /* decoding_context.rs:18 */
  uint8_t* decoded; size_t len, cap;             /* :19 */
  uint64_t offsets[3];                           /* :20 */
  uint64_t window_size;
  int has_rep[3]; sym_mode rep[3];               /* ll, cmov(offset), ml repeat decoders :22-24 */
} dctx;

#define MAX_WIN_SIZE (8ull << 20)                 /* frame.rs:44 */

static int ctx_new(dctx* c, uint64_t window) {     /* decoding_context.rs:29-47 */
  if (window > MAX_WIN_SIZE) return ZD_E_CTX_WINDOW_SIZE_TOO_BIG;
  memset(c, 0, sizeof *c);
  c->offsets[0] = 1; c->offsets[1] = 4; c->offsets[2] = 8; c->window_size = window;
  return 0;
}
static void ctx_free(dctx* c) {
  free(c->decoded); h_free(&c->huffman);
  for (int i = 0; i < 3; i++) if (c->has_rep[i] && c->rep[i].table) free(c->rep[i].table);
}
static int ctx_reserve(dctx* c, size_t extra) {
  if (c->len + extra <= c->cap) return 0;
  size_t nc = c->cap ? c->cap : 4096;
  while (nc < c->len + extra) nc *= 2;
  uint8_t* nd = (uint8_t*)realloc(c->decoded, nc);
  if (!nd) return ZD_E_NO_MEMORY;
  c->decoded = nd; c->cap = nc; return 0;
}

/* DecodingContext::decode_offset (decoding_context.rs:50-75) */
static int ctx_decode_offset(dctx* c, uint64_t offset, uint64_t ll, uint64_t* out) {
  uint64_t* o = c->offsets;
  if (offset == 0) return ZD_E_NULL_OFFSET;
  if (offset == 3 && ll == 0) {
    o[2] = o[1]; o[1] = o[0];
    if (o[0] == 0) return ZD_E_REF_PANIC;       /* usize underflow */
    o[0] -= 1;
  } else if ((offset == 3) || (offset == 2 && ll == 0)) {
    uint64_t t = o[2]; o[2] = o[1]; o[1] = o[0]; o[0] = t;
  } else if ((offset == 2) || (offset == 1 && ll == 0)) {
    uint64_t t = o[0]; o[0] = o[1]; o[1] = t;
  } else if (offset == 1) {
  } else {
    o[2] = o[1]; o[1] = o[0]; o[0] = offset - 3;
  }
  *out = o[0]; return 0;
}

/* DecodingContext::execute_sequences (decoding_context.rs:78-106) */
static int ctx_execute(dctx* c, const uint64_t* seqs, size_t nseq, const uint8_t* lits, size_t nl) {
  for (size_t i = 0; i < nseq; i++) {
    uint64_t ll = seqs[3 * i], ofv = seqs[3 * i + 1], ml = seqs[3 * i + 2];
    uint64_t off; TRY(ctx_decode_offset(c, ofv, ll, &off));
    if (ll > nl || off > c->len + ll) return ZD_E_IMPOSSIBLE_VALUE;
    TRY(ctx_reserve(c, ll + ml));
    memcpy(c->decoded + c->len, lits, ll); c->len += ll; lits += ll; nl -= ll;
    if (ml && off == 0) return ZD_E_REF_PANIC;   /* decoded[len - 0] out of bounds (D9) */
    uint8_t* d = c->decoded;
    for (uint64_t k = 0; k < ml; k++) { d[c->len] = d[c->len - off]; c->len++; }
  }
  TRY(ctx_reserve(c, nl));
  memcpy(c->decoded + c->len, lits, nl); c->len += nl;
  return 0;
}

/* ---------------- decoders/sequence.rs ---------------- */
static const uint32_t ML_BASE[53] = {           /* sequence.rs:98-152 */
  3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31,32,33,34,
  35,37,39,41,43,47,51,59,67,83,99,131,259,515,1027,2051,4099,8195,16387,32771,65539 };
static const uint8_t ML_BITS[53] = {
  0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,
  1,1,1,1,2,2,3,3,4,4,5,7,8,9,10,11,12,13,14,15,16 };
static const uint32_t LL_BASE[36] = {           /* sequence.rs:154-191 */
  0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,18,20,22,24,28,32,40,48,64,128,256,512,1024,2048,4096,
  8192,16384,32768,65536 };
static const uint8_t LL_BITS[36] = {
  0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,1,1,1,1,2,2,3,3,4,6,7,8,9,10,11,12,13,14,15,16 };

/* ---------------- sequences.rs ---------------- */
static const int16_t LL_DEFAULT[36] = {          /* sequences.rs:29-32 */
  4,3,2,2,2,2,2,2,2,2,2,2,2,1,1,1,2,2,2,2,2,2,2,2,2,3,2,1,1,1,1,1,-1,-1,-1,-1 };
static const int16_t OF_DEFAULT[29] = {          /* sequences.rs:33-35 */
  1,1,1,1,1,1,2,2,2,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,-1,-1,-1,-1,-1 };
static const int16_t ML_DEFAULT[53] = {          /* sequences.rs:36-39 */
  1,4,3,2,2,2,2,2,2,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,
  1,1,1,1,1,1,1,1,1,1,1,1,1,1,-1,-1,-1,-1,-1,-1,-1 };

typedef struct {
  size_t nseq;
  sym_mode modes[3];          /* LL, OF, ML */
  const uint8_t* bitstream; size_t bs_len;
} sequences_section;

/* Sequences::parse_num_sequences (sequences.rs:77-87), D1 kept */
static int seq_parse_num(fbp* in, size_t* out, zdo_err* e) {
  uint8_t b0, b1, b2; TRY(fbp_u8(in, &b0, e));
  if (b0 == 0) *out = 0;
  else if (b0 < 128) *out = b0;
  else if (b0 < 255) { TRY(fbp_u8(in, &b1, e)); *out = ((size_t)(b0 - 128) << 8) + b1; }
  else { TRY(fbp_u8(in, &b1, e)); TRY(fbp_u8(in, &b2, e)); *out = (size_t)b1 + ((size_t)b2 << 8) + 0x7F; }
  return 0;
}

/* Sequences::parse + parse_symbol_compression (sequences.rs:52-143) */
static int seq_parse(fbp* in, sequences_section* S, zdo_err* e) {
  memset(S, 0, sizeof *S);
  TRY(seq_parse_num(in, &S->nseq, e));
  for (int i = 0; i < 3; i++) S->modes[i].mode = M_REPEAT;
  S->bitstream = NULL; S->bs_len = 0;
  if (S->nseq == 0) return 0;
  const uint8_t* mb; TRY(fbp_slice(in, 1, &mb, e));
  if (mb[0] & 3) return fail(e, ZD_E_SEQ_RESERVED_SET, 0, 0);
  int mt[3] = { (mb[0] >> 6) & 3, (mb[0] >> 4) & 3, (mb[0] >> 2) & 3 };   /* LL, OF, ML */
  for (int i = 0; i < 3; i++) {
    S->modes[i].mode = mt[i];
    if (mt[i] == M_RLE) { TRY(fbp_u8(in, &S->modes[i].rle, e)); }
    else if (mt[i] == M_FSE) {
      const uint8_t* nd; size_t nn = in->n;
      TRY(fbp_slice(in, in->n, &nd, e));
      fwbits fw; TRY(fw_new(&fw, nd, nn, e));
      int16_t dist[MAX_SYMBOL]; size_t nsym; uint8_t al;
      TRY(parse_fse_table(&fw, &al, dist, &nsym, e));
      fse_table* t = (fse_table*)malloc(sizeof(fse_table));
      if (!t) return ZD_E_NO_MEMORY;
      int r = fse_from_distribution(al, dist, nsym, t, e);
      if (r) { free(t); return r; }
      S->modes[i].table = t;
      size_t br = (size_t)fw_bytes_read(&fw);
      in->p = nd + br; in->n = nn - br;
    }
  }
  S->bs_len = in->n;
  TRY(fbp_slice(in, in->n, &S->bitstream, e));
  return 0;
}

static void seq_free(sequences_section* S) {
  for (int i = 0; i < 3; i++) if (S->modes[i].table) { free(S->modes[i].table); S->modes[i].table = NULL; }
}

static fse_table g_predef[3];
static int g_predef_ok = 0;
static void predef_init(void) {
  if (g_predef_ok) return;
  fse_from_distribution(6, LL_DEFAULT, 36, &g_predef[0], NULL);
  fse_from_distribution(5, OF_DEFAULT, 29, &g_predef[1], NULL);
  fse_from_distribution(6, ML_DEFAULT, 53, &g_predef[2], NULL);
  g_predef_ok = 1;
}

/* Sequences::get_decoder (sequences.rs:147-187): resolved mode kept by the
 * decoder (table pointer borrowed; the resolved mode is later copied into the
 * context). code: 0 LL, 1 OF, 2 ML. */
static int seq_get_decoder(int code, const sym_mode* m, int has_prev, const sym_mode* prev, bitdec* d, sym_mode* resolved) {
  switch (m->mode) {
    case M_RLE: d->table = NULL; d->rle = m->rle; *resolved = *m; return 0;
    case M_FSE: d->table = m->table; *resolved = *m; return 0;
    case M_PREDEFINED: predef_init(); d->table = &g_predef[code]; resolved->mode = M_PREDEFINED; resolved->table = NULL; return 0;
    default:
      if (!has_prev || prev->mode == M_REPEAT) return ZD_E_NO_PREVIOUS_DECODER;
      return seq_get_decoder(code, prev, 0, NULL, d, resolved);
  }
}

static fse_table* table_dup(const fse_table* t) {
  fse_table* n = (fse_table*)malloc(sizeof *n);
  if (n) memcpy(n, t, sizeof *n);
  return n;
}

/* Sequences::decode (sequences.rs:191-237) with SequenceDecoder
 * (decoders/sequence.rs:30-93).  seqs: malloc'd triples. */
static int seq_decode(sequences_section* S, dctx* c, uint64_t** seqs_out, zdo_err* e) {
  bitdec dec[3]; sym_mode res[3];
  memset(dec, 0, sizeof dec);
  TRY(seq_get_decoder(0, &S->modes[0], c->has_rep[0], &c->rep[0], &dec[0], &res[0]));
  TRY(seq_get_decoder(1, &S->modes[1], c->has_rep[1], &c->rep[1], &dec[1], &res[1]));
  TRY(seq_get_decoder(2, &S->modes[2], c->has_rep[2], &c->rep[2], &dec[2], &res[2]));
  bwbits bs; TRY(bw_new(&bs, S->bitstream, S->bs_len, e));
  /* SequenceDecoder::initialize: LL, OF, ML (sequence.rs:59-65) */
  TRY(dec_initialize(&dec[0], &bs, e)); TRY(dec_initialize(&dec[1], &bs, e)); TRY(dec_initialize(&dec[2], &bs, e));
  uint64_t* out = (uint64_t*)malloc(3 * sizeof(uint64_t) * (S->nseq ? S->nseq : 1));
  if (!out) return ZD_E_NO_MEMORY;
  int r = 0;
  for (size_t i = 0; i < S->nseq; i++) {
    /* update_symbol_value (sequence.rs:41-55) */
    uint16_t ofc, llc, mlc;
    if ((r = dec_symbol(&dec[1], &ofc))) break;
    if ((r = dec_symbol(&dec[0], &llc))) break;
    if ((r = dec_symbol(&dec[2], &mlc))) break;
    if (llc > 35 || mlc > 52 || ofc > 31) { r = fail(e, ZD_E_SEQUENCE_CODE_MAX_EXCEEDED, 0, 0); break; }
    uint64_t v;
    if ((r = bw_take(&bs, ofc, &v, e))) break;
    uint64_t ofv = ((uint64_t)1 << ofc) + v;
    if ((r = bw_take(&bs, ML_BITS[mlc], &v, e))) break;
    uint64_t ml = ML_BASE[mlc] + v;
    if ((r = bw_take(&bs, LL_BITS[llc], &v, e))) break;
    uint64_t ll = LL_BASE[llc] + v;
    out[3 * i] = ll; out[3 * i + 1] = ofv; out[3 * i + 2] = ml;
    if (i + 1 == S->nseq) break;
    /* update_bits: LL, ML, OF (sequence.rs:80-88) */
    if ((r = dec_update(&dec[0], &bs, e))) break;
    if ((r = dec_update(&dec[2], &bs, e))) break;
    if ((r = dec_update(&dec[1], &bs, e))) break;
  }
  if (r) { free(out); return r; }
  /* context.*_repeat_decoder = Some(resolved) (sequences.rs:232-234) */
  for (int k = 0; k < 3; k++) {
    sym_mode nm = res[k];
    if (nm.mode == M_FSE) { nm.table = table_dup(nm.table); if (!nm.table) { free(out); return ZD_E_NO_MEMORY; } }
    if (c->has_rep[k] && c->rep[k].table) free(c->rep[k].table);
    c->rep[k] = nm; c->has_rep[k] = 1;
  }
  *seqs_out = out; return 0;
}

/* ---------------- block.rs ---------------- */
typedef struct {
  int type;                    /* 0 raw, 1 rle, 2 compressed */
  const uint8_t* raw; size_t raw_len;
  uint8_t byte; uint32_t repeat;
  literals_section lit; sequences_section seq;
} block_t;

static void block_free(block_t* b) {
  if (b->type == 2) { if (b->lit.has_tree) h_free(&b->lit.tree); seq_free(&b->seq); }
}

/* Block::parse (block.rs:43-72) */
static int block_parse(fbp* p, block_t* b, int* last, zdo_err* e) {
  memset(b, 0, sizeof *b);
  b->type = -1;
  const uint8_t* h; TRY(fbp_slice(p, 3, &h, e));
  uint32_t x = h[0] | (h[1] << 8) | ((uint32_t)h[2] << 16);
  *last = x & 1;
  int type = (x >> 1) & 3;
  size_t size = x >> 3;
  if (type == 0) { TRY(fbp_slice(p, size, &b->raw, e)); b->raw_len = size; b->type = 0; return 0; }
  if (type == 1) { TRY(fbp_u8(p, &b->byte, e)); b->repeat = (uint32_t)size; b->type = 1; return 0; }
  if (type == 2) {
    const uint8_t* c; TRY(fbp_slice(p, size, &c, e));
    fbp np = { c, size };
    b->type = 2;
    TRY(lit_parse(&np, &b->lit, e));
    TRY(seq_parse(&np, &b->seq, e));
    return 0;
  }
  return fail(e, ZD_E_RESERVED_BLOCK_TYPE, 0, 0);
}

/* LiteralsSection::decode (literals.rs:49-86) */
static int lit_decode(literals_section* L, dctx* c, uint8_t** out, size_t* nout, zdo_err* e) {
  if (L->type == LIT_RAW) {
    *out = (uint8_t*)malloc(L->data_len ? L->data_len : 1);
    if (!*out) return ZD_E_NO_MEMORY;
    memcpy(*out, L->data, L->data_len); *nout = L->data_len; return 0;
  }
  if (L->type == LIT_RLE) {
    *out = (uint8_t*)malloc(L->repeat ? L->repeat : 1);
    if (!*out) return ZD_E_NO_MEMORY;
    memset(*out, L->byte, L->repeat); *nout = L->repeat; return 0;
  }
  if (L->has_tree) {
    h_free(&c->huffman); c->huffman = L->tree; c->has_huffman = 1;
    L->has_tree = 0; memset(&L->tree, 0, sizeof L->tree);
  }
  if (!c->has_huffman) return fail(e, ZD_E_HUFFMAN_DECODER_MISSING, 0, 0);
  size_t cap = 1024, len = 0;
  uint8_t* res = (uint8_t*)malloc(cap);
  if (!res) return ZD_E_NO_MEMORY;
  const uint8_t* data = L->data;
  for (int s = 0; s < 4; s++) {
    size_t ss = L->jump[s];
    if (ss == 0) break;
    bwbits bs; int r = bw_new(&bs, data, ss, e);
    if (r) { free(res); return r; }
    data += ss;
    while (bs.readable != 0) {
      if (len == cap) { cap *= 2; uint8_t* nr = (uint8_t*)realloc(res, cap); if (!nr) { free(res); return ZD_E_NO_MEMORY; } res = nr; }
      r = h_decode(&c->huffman, &bs, &res[len], e);
      if (r) { free(res); return r; }
      len++;
    }
  }
  *out = res; *nout = len; return 0;
}

/* Block::decode (block.rs:74-99).  If stage_seqs is non-NULL the decoded
 * sequences/literals are handed back instead of freed. */
static int block_decode(block_t* b, dctx* c, zdo_err* e,
                        uint64_t** stage_seqs, size_t* stage_nseq, uint8_t** stage_lits, size_t* stage_nl) {
  if (b->type == 0) { TRY(ctx_reserve(c, b->raw_len)); memcpy(c->decoded + c->len, b->raw, b->raw_len); c->len += b->raw_len; return 0; }
  if (b->type == 1) { TRY(ctx_reserve(c, b->repeat)); memset(c->decoded + c->len, b->byte, b->repeat); c->len += b->repeat; return 0; }
  uint8_t* lits = NULL; size_t nl = 0;
  TRY(lit_decode(&b->lit, c, &lits, &nl, e));
  uint64_t* seqs = NULL;
  int r = seq_decode(&b->seq, c, &seqs, e);
  if (r) { free(lits); return r; }
  r = ctx_execute(c, seqs, b->seq.nseq, lits, nl);
  if (!r && stage_seqs) {
    *stage_seqs = seqs; *stage_nseq = b->seq.nseq; *stage_lits = lits; *stage_nl = nl;
    return 0;
  }
  free(seqs); free(lits);
  return r;
}

/* ---------------- frame.rs ---------------- */
#define MAGIC_ZSTD 0xFD2FB528u                 /* frame.rs:41 */
#define MAGIC_SKIP 0x184D2A50u                 /* frame.rs:42 */

typedef struct { int checksum_flag; uint64_t window, dict, fcs; } header_t;

/* Header::parse (frame.rs:111-177) + parse_window_descriptor (179-187) */
static int header_parse(fbp* in, header_t* h, zdo_err* e) {
  const uint8_t* b; TRY(fbp_slice(in, 1, &b, e));
  unsigned fhd = b[0];
  unsigned dict_flag = fhd & 3, csum = (fhd >> 2) & 1, reserved = (fhd >> 3) & 1;
  unsigned single = (fhd >> 5) & 1, fcs_flag = fhd >> 6;
  if (reserved) return fail(e, ZD_E_FRAME_RESERVED_SET, 0, 0);
  int fcs_size = -1;
  if (fcs_flag == 0 && !single) fcs_size = -1;
  else if (fcs_flag == 0 && single) fcs_size = 1;
  else fcs_size = 1 << fcs_flag;
  uint64_t window = UINT64_MAX; int has_window = 0;
  if (!single) {
    uint8_t wd; TRY(fbp_u8(in, &wd, e));
    uint64_t mantissa = wd & 7, exponent = wd >> 3;
    uint64_t base = (uint64_t)1 << (exponent + 10);
    window = base + (base / 8) * mantissa; has_window = 1;
  }
  h->dict = UINT64_MAX;
  if (dict_flag) {
    size_t dl = (size_t)1 << (dict_flag - 1);
    const uint8_t* a; TRY(fbp_slice(in, dl, &a, e));
    uint64_t v = 0; for (size_t i = 0; i < dl; i++) v |= (uint64_t)a[i] << (8 * i);
    h->dict = v;
  }
  h->fcs = UINT64_MAX;
  if (fcs_size > 0) {
    const uint8_t* a; TRY(fbp_slice(in, (size_t)fcs_size, &a, e));
    uint64_t v = 0; for (int i = 0; i < fcs_size; i++) v |= (uint64_t)a[i] << (8 * i);
    if (fcs_size == 2) v += 256;
    h->fcs = v;
  }
  if (!has_window) window = h->fcs;   /* single segment: FCS always present */
  h->window = window; h->checksum_flag = (int)csum;
  return 0;
}

typedef struct {
  int skippable; const uint8_t* skip_data; size_t skip_len;
  header_t hdr; block_t* blocks; size_t nblocks; int has_checksum; uint32_t checksum;
} frame_t;

static void frame_free(frame_t* f) {
  for (size_t i = 0; i < f->nblocks; i++) block_free(&f->blocks[i]);
  free(f->blocks); f->blocks = NULL; f->nblocks = 0;
}

/* Frame::parse (frame.rs:61-77) + ZStandard::parse (frame.rs:198-230) */
static int frame_parse(fbp* in, frame_t* f, zdo_err* e) {
  memset(f, 0, sizeof *f);
  uint32_t magic; TRY(fbp_le_u32(in, &magic, e));
  if (magic == MAGIC_ZSTD) {
    TRY(header_parse(in, &f->hdr, e));
    if (f->hdr.window > MAX_WIN_SIZE) return fail(e, ZD_E_WINDOW_SIZE_TOO_BIG, (int64_t)MAX_WIN_SIZE, (int64_t)f->hdr.window);
    size_t cap = 4;
    f->blocks = (block_t*)malloc(cap * sizeof(block_t));
    if (!f->blocks) return ZD_E_NO_MEMORY;
    for (;;) {
      if (f->nblocks == cap) {
        cap *= 2; block_t* nb = (block_t*)realloc(f->blocks, cap * sizeof(block_t));
        if (!nb) { frame_free(f); return ZD_E_NO_MEMORY; }
        f->blocks = nb;
      }
      int last = 0;
      int r = block_parse(in, &f->blocks[f->nblocks], &last, e);
      f->nblocks++;            /* keep for freeing partially parsed tables */
      if (r) { frame_free(f); return r; }
      if (last) break;
    }
    if (f->hdr.checksum_flag) {
      uint32_t cs; zdo_err tmp;
      if (fbp_le_u32(in, &cs, &tmp)) { frame_free(f); return fail(e, ZD_E_MISSING_CHECKSUM, tmp.a, tmp.b); }
      f->has_checksum = 1; f->checksum = cs;
    }
    return 0;
  }
  if ((magic ^ MAGIC_SKIP) <= 0x0F) {
    uint32_t dl; TRY(fbp_le_u32(in, &dl, e));
    TRY(fbp_slice(in, dl, &f->skip_data, e));
    f->skippable = 1; f->skip_len = dl; return 0;
  }
  return fail(e, ZD_E_UNRECOGNIZED_MAGIC, magic, 0);
}

/* Frame::decode (frame.rs:79-84) + ZStandard::decode (frame.rs:232-260);
 * the XXH64 comparison only prints in the reference (D5) and is omitted. */
static int frame_decode(frame_t* f, uint8_t** out, size_t* out_len, zdo_err* e,
                        size_t stage_block, uint64_t** ss, size_t* sn, uint8_t** sl, size_t* sln) {
  if (f->skippable) {
    *out = (uint8_t*)malloc(f->skip_len ? f->skip_len : 1);
    if (!*out) return ZD_E_NO_MEMORY;
    memcpy(*out, f->skip_data, f->skip_len); *out_len = f->skip_len; return 0;
  }
  dctx c; TRY(ctx_new(&c, f->hdr.window));
  for (size_t i = 0; i < f->nblocks; i++) {
    int r = block_decode(&f->blocks[i], &c, e,
                         (ss && i == stage_block) ? ss : NULL, sn, sl, sln);
    if (r) { ctx_free(&c); return r; }
  }
  *out = c.decoded; *out_len = c.len; c.decoded = NULL;
  ctx_free(&c);
  return 0;
}

/* ---------------- public ---------------- */
void zdo_free(void* p) { free(p); }

int zdo_frame_decode(const uint8_t* src, size_t n, size_t* consumed, uint8_t** out, size_t* out_len,
                     int* is_skippable, zdo_err* err) {
  zdo_err e0 = {0, 0, 0}; if (!err) err = &e0;
  fbp in = { src, n };
  frame_t f;
  *out = NULL; *out_len = 0;
  int r = frame_parse(&in, &f, err);
  if (consumed) *consumed = n - in.n;
  if (r) return err->code = r;
  if (is_skippable) *is_skippable = f.skippable;
  r = frame_decode(&f, out, out_len, err, 0, NULL, NULL, NULL, NULL);
  frame_free(&f);
  return err->code = r;
}

int zdo_decompress(const uint8_t* src, size_t n, int print_skippable,
                   uint8_t** out, size_t* out_len, size_t* frames, zdo_err* err) {
  zdo_err e0 = {0, 0, 0}; if (!err) err = &e0;
  size_t cap = 1 << 16, len = 0, nf = 0;
  uint8_t* res = (uint8_t*)malloc(cap);
  if (!res) return ZD_E_NO_MEMORY;
  fbp in = { src, n };
  int r = 0;
  while (in.n) {                                   /* FrameIterator::next (frame.rs:94-99) */
    frame_t f;
    r = frame_parse(&in, &f, err);
    if (r) break;
    if (f.skippable && !print_skippable) { frame_free(&f); nf++; continue; }
    uint8_t* fo = NULL; size_t fl = 0;
    r = frame_decode(&f, &fo, &fl, err, 0, NULL, NULL, NULL, NULL);
    frame_free(&f);
    if (r) break;
    if (len + fl > cap) {
      while (len + fl > cap) cap *= 2;
      uint8_t* nr = (uint8_t*)realloc(res, cap);
      if (!nr) { free(fo); r = ZD_E_NO_MEMORY; break; }
      res = nr;
    }
    memcpy(res + len, fo, fl); len += fl; free(fo); nf++;
  }
  *out = res; *out_len = len; if (frames) *frames = nf;
  return err->code = r;
}

int zdo_forward_bits(const uint8_t* d, size_t n, const uint32_t* takes, size_t nt,
                     uint64_t* vals, uint64_t* len_after, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  fwbits f; TRY(fw_new(&f, d, n, err));
  for (size_t i = 0; i < nt; i++) {
    int r = fw_take(&f, takes[i], &vals[i], err);
    if (r) { if (len_after) *len_after = f.readable; return r; }
  }
  if (len_after) *len_after = f.readable;
  return 0;
}

int zdo_backward_bits(const uint8_t* d, size_t n, const uint32_t* takes, size_t nt,
                      uint64_t* vals, uint64_t* len_before, uint64_t* len_after, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  bwbits b; TRY(bw_new(&b, d, n, err));
  if (len_before) *len_before = b.readable;
  for (size_t i = 0; i < nt; i++) {
    int r = bw_take(&b, takes[i], &vals[i], err);
    if (r) { if (len_after) *len_after = b.readable; return r; }
  }
  if (len_after) *len_after = b.readable;
  return 0;
}

int zdo_parse_fse_table(const uint8_t* d, size_t n, uint8_t* al, int16_t* dist,
                        size_t* nsym, uint64_t* bits_left, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  fwbits f; TRY(fw_new(&f, d, n, err));
  TRY(parse_fse_table(&f, al, dist, nsym, err));
  if (bits_left) *bits_left = f.readable;
  return 0;
}

int zdo_fse_from_distribution(uint8_t al, const int16_t* dist, size_t n, uint16_t* out, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  fse_table* t = (fse_table*)malloc(sizeof *t);
  if (!t) return ZD_E_NO_MEMORY;
  int r = fse_from_distribution(al, dist, n, t, err);
  if (!r) for (size_t i = 0; i < ((size_t)1 << al); i++) {
    out[3 * i] = t->t[i].output; out[3 * i + 1] = t->t[i].baseline; out[3 * i + 2] = t->t[i].bits;
  }
  free(t); return r;
}

static void table_from_u16(const uint16_t* table, uint8_t al, fse_table* t) {
  for (size_t i = 0; i < ((size_t)1 << al); i++) {
    t->t[i].output = table[3 * i]; t->t[i].baseline = table[3 * i + 1]; t->t[i].bits = table[3 * i + 2];
  }
  t->al = al;
}

int zdo_fse_decode(const uint16_t* table, uint8_t al, const uint8_t* stream, size_t n,
                   size_t nsym, uint16_t* syms, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  if (al > MAX_AL) return ZD_E_LARGE_ACCURACY_LOG;
  fse_table t; table_from_u16(table, al, &t);
  bitdec d; memset(&d, 0, sizeof d); d.table = &t;
  bwbits bs; TRY(bw_new(&bs, stream, n, err));
  TRY(dec_initialize(&d, &bs, err));
  for (size_t i = 0; i < nsym; i++) { TRY(dec_symbol(&d, &syms[i])); TRY(dec_update(&d, &bs, err)); }
  return 0;
}

int zdo_alternating_decode(const uint16_t* table, uint8_t al, const uint8_t* stream, size_t n,
                           size_t nsym, uint16_t* syms, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  if (al > MAX_AL) return ZD_E_LARGE_ACCURACY_LOG;
  fse_table t; table_from_u16(table, al, &t);
  altdec d; memset(&d, 0, sizeof d); d.a.table = &t; d.b.table = &t;
  bwbits bs; TRY(bw_new(&bs, stream, n, err));
  TRY(alt_initialize(&d, &bs, err));
  for (size_t i = 0; i < nsym; i++) { TRY(alt_symbol(&d, &syms[i])); TRY(alt_update(&d, &bs, err)); }
  return 0;
}

static int h_decode_all(const htree* t, const uint8_t* stream, size_t n, uint8_t* out, size_t cap, size_t* nout, zdo_err* err) {
  bwbits bs; TRY(bw_new(&bs, stream, n, err));
  size_t k = 0;
  while (bs.readable) {
    if (k == cap) return ZD_E_DST_TOO_SMALL;
    TRY(h_decode(t, &bs, &out[k], err)); k++;
  }
  *nout = k; return 0;
}

int zdo_huffman_weights_decode(const uint8_t* weights, size_t nw, const uint8_t* stream, size_t n,
                               uint8_t* out, size_t cap, size_t* nout, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  htree t = {0};
  int r = h_from_weights(weights, nw, &t);
  if (!r) r = h_decode_all(&t, stream, n, out, cap, nout, err);
  h_free(&t); return err->code = r;
}

int zdo_huffman_parse_decode(const uint8_t* desc, size_t dn, size_t* consumed,
                             const uint8_t* stream, size_t n,
                             uint8_t* out, size_t cap, size_t* nout, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  fbp in = { desc, dn };
  htree t = {0};
  int r = h_parse(&in, &t, err);
  if (consumed) *consumed = dn - in.n;
  if (!r) r = h_decode_all(&t, stream, n, out, cap, nout, err);
  h_free(&t); return err->code = r;
}

int zdo_huffman_widths(const uint8_t* desc, size_t dn, uint8_t* widths, size_t* nwidths,
                       size_t* consumed, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  fbp in = { desc, dn };
  uint8_t* w = NULL; size_t nw = 0;
  int r = h_parse_weights(&in, &w, &nw, err);
  if (consumed) *consumed = dn - in.n;
  if (r) return err->code = r;
  r = h_widths_from_weights(w, nw, widths);
  *nwidths = nw + 1;
  free(w); return err->code = r;
}

int zdo_execute_sequences(const uint64_t* seqs, size_t nseq, const uint8_t* lits, size_t nl,
                          uint8_t* out, size_t cap, size_t* nout, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  dctx c; TRY(ctx_new(&c, 0x42));
  int r = ctx_execute(&c, seqs, nseq, lits, nl);
  if (!r) {
    if (c.len > cap) r = ZD_E_DST_TOO_SMALL;
    else { memcpy(out, c.decoded, c.len); *nout = c.len; }
  }
  ctx_free(&c); return err->code = r;
}

int zdo_header_parse(const uint8_t* d, size_t n, uint64_t out[4], size_t* consumed, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  fbp in = { d, n };
  header_t h;
  int r = header_parse(&in, &h, err);
  if (consumed) *consumed = n - in.n;
  if (r) return err->code = r;
  out[0] = (uint64_t)h.checksum_flag; out[1] = h.window; out[2] = h.dict; out[3] = h.fcs;
  return 0;
}

int zdo_block_stages(const uint8_t* src, size_t n, size_t block_index,
                     uint64_t** seqs, size_t* nseq, uint8_t** lits, size_t* nlits, zdo_err* err) {
  zdo_err e0; if (!err) err = &e0; err->code = 0;
  fbp in = { src, n };
  frame_t f;
  *seqs = NULL; *lits = NULL; *nseq = 0; *nlits = 0;
  TRY(frame_parse(&in, &f, err));
  if (f.skippable || block_index >= f.nblocks || f.blocks[block_index].type != 2) { frame_free(&f); return ZD_E_INVALID_ARG; }
  uint8_t* o = NULL; size_t ol = 0;
  int r = frame_decode(&f, &o, &ol, err, block_index, seqs, nseq, lits, nlits);
  free(o); frame_free(&f);
  return err->code = r;
}
