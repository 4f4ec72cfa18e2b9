/*
 * norm_fec_oracle.h -- CPU restatement of NORM's FEC codecs (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity checker for the MI355X path, not part of the product.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (norm_amd/_lib/libnfec.so) never links or calls it.
 *
 * Each routine restates the reference algorithm it cites (paths relative to the
 * USNavalResearchLaboratory/norm tree).  Pinning status (see DESIGN.md "Oracle"):
 *   - GF(2^8) arithmetic (RS8 gf_exp/gf_log/gf_mul_table and the MDP GEXP/GMULT/GINV
 *     tables) is PINNED against tests/golden/galois_tables.json, produced by compiling
 *     the reference's own src/common/galois.cpp (oracle/ref/Makefile).
 *   - The RS8/RS16 generator build, incremental encode, Gauss-Jordan decode and the MDP
 *     LFSR / Forney decode are restated from source but their outputs are UNPINNED by
 *     any reference-produced vector: the reference codec translation units include
 *     protolib headers (protoDefs.h / protoDebug.h / protokit.h) that are absent from
 *     this image (protolib is an empty, un-vendored submodule), so they are
 *     unbuildable here, and the reference ships no known-answer FEC vectors
 *     (src/common/fecTest.cpp only round-trips).
 */
#ifndef NORM_FEC_ORACLE_H
#define NORM_FEC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- field tables (normEncoderRS8.cpp:182-242, normEncoderRS16.cpp:181-241) ---- */
void orc_gf8_tables(uint8_t exp_out[510], int32_t log_out[256], uint8_t inv_out[256]);
void orc_gf8_mul_table(uint8_t out[65536]);
void orc_gf16_tables(uint16_t* exp_out /*131070*/, int32_t* log_out /*65536*/, uint16_t* inv_out /*65536*/);
/* galois.cpp constant tables, restated (galois.cpp:37,58,95) */
void orc_galois_tables(uint8_t ginv[256], uint8_t gexp[512], uint8_t gmult[65536]);

/* ---- RS8 / RS16 generator (normEncoderRS8.cpp:400-462) ----
 * enc_out receives the full n x k systematic matrix, row-major (n = k + m).
 * RS8: bytes; RS16: uint16 elements.  Returns 0 on success, -1 when k+m exceeds the field. */
int orc_rs8_generator(unsigned k, unsigned m, uint8_t* enc_out);
int orc_rs16_generator(unsigned k, unsigned m, uint16_t* enc_out);

/* ---- RS incremental encode (normEncoderRS8.cpp:473-483): parity[i] ^= enc[k+i][seg] * data ---- */
void orc_rs8_encode(const uint8_t* enc, unsigned k, unsigned m, unsigned vec,
                    unsigned segment_id, const uint8_t* data, uint8_t** parity);
void orc_rs16_encode(const uint16_t* enc, unsigned k, unsigned m, unsigned vec,
                     unsigned segment_id, const uint8_t* data, uint8_t** parity);

/* ---- RS decode (normEncoderRS8.cpp:652-757, Gauss-Jordan :766-889) ----
 * vectors: [0,numData) source, [numData,numData+m) parity, like NORM's block segment list.
 * Returns erasure_count, or 0 on singular matrix -- exactly the reference convention. */
int orc_rs8_decode(const uint8_t* enc, unsigned k, unsigned m, unsigned vec, uint8_t** vectors,
                   unsigned num_data, unsigned erasure_count, const unsigned* erasure_locs);
int orc_rs16_decode(const uint16_t* enc, unsigned k, unsigned m, unsigned vec, uint8_t** vectors,
                    unsigned num_data, unsigned erasure_count, const unsigned* erasure_locs);

/* ---- MDP (normEncoderMDP.cpp) ---- */
int orc_mdp_generator_poly(unsigned m, uint8_t* gen_poly_out /* m+1 */);         /* :102-170 */
void orc_mdp_encode(const uint8_t* gen_poly, unsigned m, unsigned vec,
                    const uint8_t* data, uint8_t** parity, uint8_t* scratch);    /* :178-211 */
int orc_mdp_decode(unsigned m, unsigned vec, uint8_t** vectors, unsigned num_data,
                   unsigned erasure_count, const unsigned* erasure_locs);       /* :333-430 */

/* ---- contiguous-block conveniences used by the tests ----
 * block layout: slot s at block + s*seg_stride, slots [0,num_data) source then m parity. */
int orc_encode_blocks(int fec_kind, unsigned k, unsigned m, unsigned vec, uint8_t* blocks,
                      uint64_t block_stride, unsigned seg_stride, const uint16_t* num_data,
                      unsigned nblocks);
int orc_decode_blocks(int fec_kind, unsigned k, unsigned m, unsigned vec, uint8_t* blocks,
                      uint64_t block_stride, unsigned seg_stride, const uint16_t* num_data,
                      const uint16_t* erasure_locs, unsigned erasure_stride,
                      const uint16_t* erasure_counts, int32_t* status, unsigned nblocks);

/* ---- synthetic workload ---- */
uint64_t orc_splitmix64_mix(uint64_t z);
void orc_fill_segment(uint64_t seed, uint64_t block, uint32_t seg, uint8_t* out, unsigned nbytes);
unsigned orc_erasure_pattern(uint64_t seed, uint64_t block, unsigned range, unsigned count,
                             uint16_t* out_sorted);

/* ---- CPU baseline timing (C1): returns wall seconds for encode and decode ----
 * threads independent workers, each with its own blocks; bounded sample of nblocks. */
int orc_bench_rs8(unsigned k, unsigned m, unsigned vec, unsigned nblocks, unsigned erasures,
                  unsigned threads, uint64_t seed, double* t_encode, double* t_decode,
                  uint64_t* bad_blocks);

#ifdef __cplusplus
}
#endif
#endif
