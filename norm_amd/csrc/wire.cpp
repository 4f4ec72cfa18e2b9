// wire.cpp -- the NORM wire-format pieces on the FEC path (host only, no GPU):
// FEC Object Transmission Information header extensions, FEC payload IDs and the codec
// selection rules a sender and a receiver apply to them.
//
// Reference layouts (USNavalResearchLaboratory/norm include/normMessage.h):
//   NormHeaderExtension        :324-389  byte 0 type (FTI = 64), byte 1 length in 32-bit words
//   NormFtiExtension2 (fec 2)  :785-839  16 bytes: obj size MSB16 @2, LSB32 @4, m @8, G @9,
//                                        segment size @10, ndata @12, nparity @14
//   NormFtiExtension5 (fec 5)  :898-942  12 bytes: obj size MSB16 @2, LSB32 @4, segment size @8,
//                                        ndata (u8) @10, nparity (u8) @11
//   NormFtiExtension129        :977-1029 16 bytes: obj size MSB16 @2, LSB32 @4, instance @8,
//                                        segment size @10, ndata @12, nparity @14
//   NormPayloadId              :396-567  fec 2/m=8 and fec 5: block<<8 | symbol (u32);
//                                        fec 2/m=16: block16, symbol16; fec 129: block32,
//                                        block length16, symbol16
// Codec selection: sender src/common/normSession.cpp:764-883, receiver src/common/normNode.cpp:290-356.
// All multi-byte fields are big-endian (network order).
#include <cstdint>
#include <cstring>

#include "nfec.h"

namespace {

void put16(uint8_t* p, uint16_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
void put32(uint8_t* p, uint32_t v)
{
    put16(p, (uint16_t)(v >> 16));
    put16(p + 2, (uint16_t)v);
}
uint16_t get16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t get32(const uint8_t* p) { return ((uint32_t)get16(p) << 16) | get16(p + 2); }

constexpr uint8_t kFti = 64;        // NormHeaderExtension::FTI
constexpr uint32_t kStreamHdr = 8;  // NormDataMsg::GetStreamPayloadHeaderLength() (PAYLOAD_DATA_OFFSET)

}  // namespace

extern "C" {

int nfec_fti_write(const nfec_fti* f, void* ext, size_t cap)
{
    if (!f || !ext) return NFEC_EINVAL;
    if (f->object_size >> 48) return NFEC_EINVAL;  // NormObjectSize is 48 bits
    uint8_t* b = static_cast<uint8_t*>(ext);
    const size_t len = f->fec_id == 5 ? 12 : 16;
    if (f->fec_id != 2 && f->fec_id != 5 && f->fec_id != 129) return NFEC_EINVAL;
    if (cap < len) return NFEC_EINVAL;
    if (f->fec_id == 5 && (f->num_data > 255 || f->num_parity > 255)) return NFEC_ERANGE;  // u8 fields
    std::memset(b, 0, len);
    b[0] = kFti;
    b[1] = (uint8_t)(len / 4);
    put16(b + 2, (uint16_t)(f->object_size >> 32));
    put32(b + 4, (uint32_t)f->object_size);
    switch (f->fec_id) {
    case 2:
        b[8] = f->fec_m;
        b[9] = f->fec_group_size;
        put16(b + 10, f->segment_size);
        put16(b + 12, f->num_data);
        put16(b + 14, f->num_parity);
        break;
    case 5:
        put16(b + 8, f->segment_size);
        b[10] = (uint8_t)f->num_data;
        b[11] = (uint8_t)f->num_parity;
        break;
    default:  // 129
        put16(b + 8, f->instance_id);
        put16(b + 10, f->segment_size);
        put16(b + 12, f->num_data);
        put16(b + 14, f->num_parity);
        break;
    }
    return (int)len;
}

int nfec_fti_read(uint8_t fec_id, const void* ext, size_t len, nfec_fti* out)
{
    if (!ext || !out) return NFEC_EINVAL;
    const uint8_t* b = static_cast<const uint8_t*>(ext);
    const size_t need = fec_id == 5 ? 12 : 16;
    if (fec_id != 2 && fec_id != 5 && fec_id != 129) return NFEC_EINVAL;
    if (len < need || b[0] != kFti || (size_t)b[1] * 4 < need) return NFEC_EINVAL;
    std::memset(out, 0, sizeof(*out));
    out->fec_id = fec_id;
    out->object_size = ((uint64_t)get16(b + 2) << 32) | get32(b + 4);
    switch (fec_id) {
    case 2:
        out->fec_m = b[8];
        out->fec_group_size = b[9];
        out->segment_size = get16(b + 10);
        out->num_data = get16(b + 12);
        out->num_parity = get16(b + 14);
        break;
    case 5:
        out->fec_m = 8;
        out->fec_group_size = 1;  // one symbol per packet, implied by fec_id 5 and 129
        out->segment_size = get16(b + 8);
        out->num_data = b[10];
        out->num_parity = b[11];
        break;
    default:
        out->fec_m = 8;
        out->fec_group_size = 1;
        out->instance_id = get16(b + 8);
        out->segment_size = get16(b + 10);
        out->num_data = get16(b + 12);
        out->num_parity = get16(b + 14);
        break;
    }
    return (int)need;
}

int nfec_payload_id_length(uint8_t fec_id)
{
    return fec_id == 2 || fec_id == 5 ? 4 : fec_id == 129 ? 8 : 0;  // NormPayloadId::GetLength
}

int nfec_payload_id_write(uint8_t fec_id, uint8_t fec_m, uint32_t block_id, uint16_t symbol_id, uint16_t block_len,
                          void* out)
{
    if (!out) return NFEC_EINVAL;
    uint8_t* b = static_cast<uint8_t*>(out);
    switch (fec_id) {
    case 2:
        if (fec_m == 8) {
            put32(b, (block_id << 8) | (symbol_id & 0xff));
        } else if (fec_m == 16) {
            put16(b, (uint16_t)block_id);
            put16(b + 2, symbol_id);
        } else {
            return NFEC_EINVAL;
        }
        return 4;
    case 5:
        put32(b, (block_id << 8) | (symbol_id & 0xff));
        return 4;
    case 129:
        put32(b, block_id);
        put16(b + 4, block_len);
        put16(b + 6, symbol_id);
        return 8;
    default:
        return NFEC_EINVAL;
    }
}

int nfec_payload_id_read(uint8_t fec_id, uint8_t fec_m, const void* in, uint32_t* block_id, uint16_t* symbol_id,
                         uint16_t* block_len)
{
    if (!in || !block_id || !symbol_id) return NFEC_EINVAL;
    const uint8_t* b = static_cast<const uint8_t*>(in);
    uint16_t blen = 0;
    switch (fec_id) {
    case 2:
        if (fec_m == 8) {
            const uint32_t v = get32(b);
            *block_id = 0x00ffffffu & (v >> 8);
            *symbol_id = (uint16_t)(v & 0xff);
        } else if (fec_m == 16) {
            *block_id = get16(b);
            *symbol_id = get16(b + 2);
        } else {
            return NFEC_EINVAL;
        }
        break;
    case 5: {
        const uint32_t v = get32(b);
        *block_id = 0x00ffffffu & (v >> 8);
        *symbol_id = (uint16_t)(v & 0xff);
        break;
    }
    case 129:
        *block_id = get32(b);
        blen = get16(b + 4);
        *symbol_id = get16(b + 6);
        break;
    default:
        return NFEC_EINVAL;
    }
    if (block_len) *block_len = blen;
    return nfec_payload_id_length(fec_id);
}

int nfec_sender_codec(uint16_t num_data, uint16_t num_parity, uint8_t fec_id_pref, int assume_mdp, int* kind,
                      uint8_t* fec_id, uint8_t* fec_m)
{
    if (!kind || !fec_id || !fec_m) return NFEC_EINVAL;
    const uint32_t block = (uint32_t)num_data + num_parity;
    if (num_parity == 0) {
        // no parity: no encoder is created, the RS8 fec_id is advertised whatever the block
        // size or ASSUME_MDP_FEC (normSession.cpp:890-898)
        *kind = 0;
        *fec_id = fec_id_pref ? fec_id_pref : 5;
        *fec_m = 8;
    } else if (block <= 255) {
        if (assume_mdp) {
            *kind = NFEC_MDP;
            *fec_id = 129;
        } else {
            *kind = NFEC_RS8;
            *fec_id = fec_id_pref ? fec_id_pref : 5;
        }
        *fec_m = 8;
    } else {
        *kind = NFEC_RS16;
        *fec_id = 2;
        *fec_m = 16;
    }
    return NFEC_OK;
}

int nfec_receiver_codec(uint8_t fec_id, uint8_t fec_m, uint16_t instance_id, int assume_mdp, int* kind)
{
    if (!kind) return NFEC_EINVAL;
    switch (fec_id) {
    case 2:
        if (fec_m == 8) *kind = NFEC_RS8;
        else if (fec_m == 16) *kind = NFEC_RS16;
        else return NFEC_ENOTSUP;  // "unsupported fecId=2 'm' value"
        return NFEC_OK;
    case 5:
        *kind = NFEC_RS8;
        return NFEC_OK;
    case 129:
        if (assume_mdp) {
            *kind = NFEC_MDP;
            return NFEC_OK;
        }
        if (instance_id == 0) {
            *kind = NFEC_RS8;
            return NFEC_OK;
        }
        return NFEC_ENOTSUP;  // "unknown fecId=129 instanceId"
    default:
        return NFEC_ENOTSUP;
    }
}

uint32_t nfec_vector_size(uint16_t segment_size) { return (uint32_t)segment_size + kStreamHdr; }

}  // extern "C"
