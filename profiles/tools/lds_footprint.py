"""LDS bytes per document of a paged launch (mirror of csrc/mt_paged.h paged_layout) and the
documents per CU they allow (160 KB LDS per CU on gfx950).
    python profiles/tools/lds_footprint.py PP UT PH [overlap_bytes] [hm]
hm: the tier keeps the page metadata in HBM (none in LDS; chunk sums and a 64-position
observer-length cache instead of pvl)"""
import sys

MT_PG_SLOTS, MT_LV, META, LDS_CU = 64, 8, 12, 160 * 1024


def pcnt_bytes(B):   # mt_engine.h pcnt_off(B, MT_LV): levels 0-1 B each, level l >= 2 B / 4^(l-1) + 8
    return 2 * B + sum((B >> (2 * (l - 1))) + 8 for l in range(2, MT_LV))


def paged_lds(PP, UT, PH, ob=4, hm=0, gen_words=0):
    o = 16 * MT_PG_SLOTS * 2 + ob * MT_PG_SLOTS
    o += 16 * UT + ((ob * UT + 7) & ~7)
    o += 8 * (PH + 1) + (0 if hm else META * PP) + ((2 * UT + 3) & ~3)
    o += 8 * ((PP + 63) // 64) + 256 if hm else 4 * PP   # chunk sums + obs cache, or pvl (r5)
    o += 64 * 4 + MT_LV * 4 * 2 + 4 * gen_words + 2 * PP + 2 * 16 + MT_LV * 16 + 16
    o += pcnt_bytes(PP) - PP
    return (o + 15) & ~15


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    b = paged_lds(*a)
    print(b, LDS_CU // b)
