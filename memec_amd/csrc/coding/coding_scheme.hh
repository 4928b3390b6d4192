// coding_scheme.hh — enum CodingScheme, same values as the reference
// (common/coding/coding_scheme.hh:4-13) so configs and callers are unchanged.
#ifndef MEMEC_AMD_CODING_SCHEME_HH
#define MEMEC_AMD_CODING_SCHEME_HH

enum CodingScheme {
    CS_UNDEFINED,
    CS_RAID0,
    CS_RAID1,
    CS_RAID5,
    CS_RS,
    CS_RDP,
    CS_EVENODD,
    CS_CAUCHY
};

#endif
