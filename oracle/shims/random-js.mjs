// TEST INFRASTRUCTURE ONLY: stand-in for the test-only npm dependency random-js@1 (absent
// here; packages/dds/merge-tree/package.json:89).  Restates the published algorithms it is
// used for: the MT19937 engine (Matsumoto & Nishimura, init_by_array seeding) and
// random-js v1 `integer(min, max)` (mask for 2^k-1 ranges, else rejection sampling).
function mt19937() {
    const mt = new Int32Array(624);
    let index = 625;
    function next() {
        if (index >= 624) { refresh(); index = 0; }
        let y = mt[index++];
        y ^= y >>> 11;
        y ^= (y << 7) & 0x9d2c5680;
        y ^= (y << 15) & 0xefc60000;
        return y ^ (y >>> 18);
    }
    function refresh() {
        let k = 0, tmp = 0;
        for (; k < 227; ++k) {
            tmp = (mt[k] & 0x80000000) | (mt[k + 1] & 0x7fffffff);
            mt[k] = mt[k + 397] ^ (tmp >>> 1) ^ ((tmp & 0x1) ? 0x9908b0df : 0);
        }
        for (; k < 623; ++k) {
            tmp = (mt[k] & 0x80000000) | (mt[k + 1] & 0x7fffffff);
            mt[k] = mt[k - 227] ^ (tmp >>> 1) ^ ((tmp & 0x1) ? 0x9908b0df : 0);
        }
        tmp = (mt[623] & 0x80000000) | (mt[0] & 0x7fffffff);
        mt[623] = mt[396] ^ (tmp >>> 1) ^ ((tmp & 0x1) ? 0x9908b0df : 0);
    }
    function seed(initial) {
        let previous = 0;
        mt[0] = previous = initial | 0;
        for (let i = 1; i < 624; i = (i + 1) | 0) {
            mt[i] = previous = (Math.imul((previous ^ (previous >>> 30)), 0x6c078965) + i) | 0;
        }
        index = 624;
    }
    next.seed = (s) => { seed(s); return next; };
    next.seedWithArray = (source) => {
        next.seed(0x012bd6aa);
        let i = 1, j = 0;
        const len = source.length;
        let k = Math.max(len, 624) | 0;
        let previous = mt[0] | 0;
        for (; (k | 0) > 0; --k) {
            mt[i] = previous = ((mt[i] ^ Math.imul((previous ^ (previous >>> 30)), 0x0019660d)) + (source[j] | 0) + (j | 0)) | 0;
            i = (i + 1) | 0; ++j;
            if ((i | 0) > 623) { mt[0] = mt[623]; i = 1; }
            if (j >= len) { j = 0; }
        }
        for (k = 623; (k | 0) > 0; --k) {
            mt[i] = previous = ((mt[i] ^ Math.imul((previous ^ (previous >>> 30)), 0x5d588b65)) - i) | 0;
            i = (i + 1) | 0;
            if ((i | 0) > 623) { mt[0] = mt[623]; i = 1; }
        }
        mt[0] = 0x80000000;
        index = 624;
        return next;
    };
    return next;
}
function integer(min, max) {
    const range = max - min;
    if (range === 0) { return () => min; }
    const ext = range + 1;
    if (((range + 1) & range) === 0 && range <= 0xffffffff) {
        return (engine) => ((engine() & range) >>> 0) + min;
    }
    const maximum = ext * Math.floor(0x100000000 / ext);
    return (engine) => {
        let v;
        do { v = engine() >>> 0; } while (v >= maximum);
        return (v % ext) + min;
    };
}
export default { engines: { mt19937 }, integer };
