// coding_params.hh — CodingParams with the reference's accessors
// (common/coding/coding_params.hh:7-173): RS / Cauchy keep k in slot 0 and
// m in slot 1; the XOR codes keep n in slot 0.
#ifndef MEMEC_AMD_CODING_PARAMS_HH
#define MEMEC_AMD_CODING_PARAMS_HH

#include <stdint.h>

#include "coding_scheme.hh"

class CodingParams {
public:
    CodingParams() : scheme_(CS_UNDEFINED) { p_[0] = p_[1] = p_[2] = 0; }

    void setScheme(CodingScheme s) { scheme_ = s; }
    void setN(uint32_t n) { if (isXor()) p_[0] = n; }
    void setK(uint32_t k) { if (isMatrix()) p_[0] = k; }
    void setM(uint32_t m) { if (isMatrix()) p_[1] = m; }
    void setW(uint32_t w) { if (isMatrix()) p_[2] = w; }

    uint32_t getN() { return isXor() ? p_[0] : 0; }
    uint32_t getK() {
        switch (scheme_) {
            case CS_RAID5: return p_[0] - 1;
            case CS_RDP:
            case CS_EVENODD: return p_[0] - 2;
            case CS_RS:
            case CS_CAUCHY: return p_[0];
            default: return 0;
        }
    }
    uint32_t getM() { return isMatrix() ? p_[1] : 0; }
    uint32_t getW() { return isMatrix() ? p_[2] : 0; }
    uint32_t getRS_K() { return 0; }
    uint32_t getRS_M() { return 0; }

    uint32_t getDataChunkCount() {
        switch (scheme_) {
            case CS_RAID0: return getN();
            case CS_RAID1: return 1;
            case CS_RAID5: return getN() - 1;
            case CS_RDP:
            case CS_EVENODD: return getN() - 2;
            case CS_RS:
            case CS_CAUCHY: return getK();
            default: return 0;
        }
    }
    uint32_t getParityChunkCount() {
        switch (scheme_) {
            case CS_RAID0: return 0;
            case CS_RAID1: return getN() - 1;
            case CS_RAID5: return 1;
            case CS_RDP:
            case CS_EVENODD: return 2;
            case CS_RS:
            case CS_CAUCHY: return getM();
            default: return 0;
        }
    }
    uint32_t getChunkCount() { return getDataChunkCount() + getParityChunkCount(); }

private:
    bool isMatrix() const { return scheme_ == CS_RS || scheme_ == CS_CAUCHY; }
    bool isXor() const {
        return scheme_ == CS_RAID0 || scheme_ == CS_RAID1 || scheme_ == CS_RAID5 || scheme_ == CS_RDP ||
               scheme_ == CS_EVENODD;
    }
    CodingScheme scheme_;
    uint32_t p_[3];
};

#endif
