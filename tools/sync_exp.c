/* Experiment (not product code): how fast does a speculative FSE sequence
 * decoder, started at an arbitrary bit position with arbitrary states,
 * fall onto the true (position, LL, OF, ML states) trajectory of a block?
 * Uses the oracle's parsers and tables (test infrastructure).
 *   gcc -O2 -o /tmp/sync_exp tools/sync_exp.c && /tmp/sync_exp file.zst [starts]
 * Per block: the true trajectory is recorded (bit position at the start of
 * every sequence and the three states); then `starts` speculative decoders
 * begin at evenly spread bit positions with states 0, and the number of
 * steps until they hit a true (pos, states) point is histogrammed. */
#include <stdio.h>
#include "../oracle/zd_oracle.c"

static uint64_t spec_take(const bwbits* b, uint64_t pos, unsigned len) {
  /* bits [8n-pos-len, 8n-pos) like bw_take; 0 when out of range */
  if (b->nbytes * 8 < pos + len || len == 0) return 0;
  return le_bits(b->d, b->nbytes, b->nbytes * 8 - pos - len, len);
}

static long hist[16];
static long nsync = 0, nfail = 0, total_steps = 0, total_seqs = 0;

static void run_block(sequences_section* S, dctx* c, int starts) {
  bitdec dec[3]; sym_mode res[3];
  memset(dec, 0, sizeof dec);
  if (seq_get_decoder(0, &S->modes[0], c->has_rep[0], &c->rep[0], &dec[0], &res[0])) return;
  if (seq_get_decoder(1, &S->modes[1], c->has_rep[1], &c->rep[1], &dec[1], &res[1])) return;
  if (seq_get_decoder(2, &S->modes[2], c->has_rep[2], &c->rep[2], &dec[2], &res[2])) return;
  if (!dec[0].table || !dec[1].table || !dec[2].table) return;
  bwbits bs; zdo_err e;
  if (bw_new(&bs, S->bitstream, S->bs_len, &e)) return;
  if (dec_initialize(&dec[0], &bs, &e) || dec_initialize(&dec[1], &bs, &e) || dec_initialize(&dec[2], &bs, &e)) return;
  size_t n = S->nseq, nbits = S->bs_len * 8;
  int64_t* at = malloc(sizeof(int64_t) * (nbits + 1));
  uint32_t* tst = malloc(sizeof(uint32_t) * n);
  for (size_t p = 0; p <= nbits; p++) at[p] = -1;
  for (size_t i = 0; i < n; i++) {
    at[bs.pos] = (int64_t)i;
    tst[i] = (uint32_t)dec[0].cur | ((uint32_t)dec[2].cur << 10) | ((uint32_t)dec[1].cur << 20);
    uint16_t ofc = dec[1].table->t[dec[1].cur].output, llc = dec[0].table->t[dec[0].cur].output,
             mlc = dec[2].table->t[dec[2].cur].output;
    dec[0].has_next = dec[1].has_next = dec[2].has_next = 0;
    uint64_t v;
    if (bw_take(&bs, ofc, &v, &e) || bw_take(&bs, ML_BITS[mlc], &v, &e) || bw_take(&bs, LL_BITS[llc], &v, &e)) break;
    if (i + 1 == n) break;
    if (dec_update(&dec[0], &bs, &e) || dec_update(&dec[2], &bs, &e) || dec_update(&dec[1], &bs, &e)) break;
  }
  total_seqs += n;
  if (getenv("AL_HIST")) { printf("al %d %d %d n %zu\n", dec[0].table->al, dec[1].table->al, dec[2].table->al, n); free(at); free(tst); return; }
  const fse_table *TL = dec[0].table, *TO = dec[1].table, *TM = dec[2].table;
  for (int s = 1; s < starts; s++) {
    uint64_t pos = (uint64_t)s * nbits / starts;
    uint32_t sl = 0, so = 0, sm = 0;
    long steps = 0;
    if (getenv("SYNC_CHECK")) {   /* sanity: start on the true trajectory, one step off the check */
      size_t i0 = (size_t)s * (n - 2) / starts;
      for (pos = 0; pos <= nbits && at[pos] != (int64_t)i0; pos++) ;
      sl = tst[i0] & 1023; sm = (tst[i0] >> 10) & 1023; so = tst[i0] >> 20;
    }
    int ok = 0;
    while (pos < nbits && steps < 100000) {
      if ((steps || !getenv("SYNC_CHECK")) && at[pos] >= 0 && tst[at[pos]] == (sl | (sm << 10) | (so << 20))) { ok = 1; break; }
      uint16_t ofc = TO->t[so].output, llc = TL->t[sl].output, mlc = TM->t[sm].output;
      if (ofc > 31) ofc = 31;
      if (llc > 35) llc = 35;
      if (mlc > 52) mlc = 52;
      pos += ofc + ML_BITS[mlc] + LL_BITS[llc];
      unsigned bl = TL->t[sl].bits, bm = TM->t[sm].bits, bo = TO->t[so].bits;
      uint64_t vl = spec_take(&bs, pos, bl); pos += bl;
      uint64_t vm = spec_take(&bs, pos, bm); pos += bm;
      uint64_t vo = spec_take(&bs, pos, bo); pos += bo;
      sl = (uint32_t)((TL->t[sl].baseline + vl) & ((1u << TL->al) - 1));
      sm = (uint32_t)((TM->t[sm].baseline + vm) & ((1u << TM->al) - 1));
      so = (uint32_t)((TO->t[so].baseline + vo) & ((1u << TO->al) - 1));
      steps++;
    }
    if (ok) {
      nsync++; total_steps += steps;
      int b = 0; while ((1L << b) <= steps && b < 15) b++;
      hist[b]++;
    } else nfail++;
  }
  free(at); free(tst);
}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
  uint8_t* d = malloc(n); fread(d, 1, n, f); fclose(f);
  int starts = argc > 2 ? atoi(argv[2]) : 16;
  fbp in = { d, (size_t)n };
  while (in.n) {
    frame_t fr; zdo_err e;
    if (frame_parse(&in, &fr, &e)) break;
    dctx c; ctx_new(&c, fr.hdr.window);
    for (size_t i = 0; i < fr.nblocks; i++) {
      block_t* b = &fr.blocks[i];
      if (b->type == 2 && b->seq.nseq > 256) run_block(&b->seq, &c, starts);
      block_decode(b, &c, &e, NULL, NULL, NULL, NULL);
    }
    ctx_free(&c); frame_free(&fr);
  }
  printf("seqs %ld  sync %ld  fail %ld  mean steps %.1f\n", total_seqs, nsync, nfail, nsync ? (double)total_steps / nsync : 0);
  for (int b = 0; b < 16; b++) if (hist[b]) printf("  < %6ld steps: %ld\n", 1L << b, hist[b]);
  return 0;
}
