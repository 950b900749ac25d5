/* kmer_map.js — KmerMap: a Map over a packed native result, built lazily.
 *
 * readFile() resolves to the reference's Map<kmer, count> in first-occurrence
 * order (lib/kmers.js:76, :95, :178).  Inserting ~2 M string keys into a V8
 * Map costs ~1 us each on node 12 (SURVEY.md §6: ~1.2 us/entry), i.e. seconds
 * at C2 against ~1 ms on the GPU.  KmerMap extends Map (instanceof Map, every
 * Map method) but keeps the counter's packed result -- one Latin-1 string of
 * all keys, offsets, counts -- and builds nothing up front:
 *   - iteration (for..of, keys(), values(), entries(), forEach, spread) walks
 *     the packed entries in order, cutting each key out of the one string;
 *   - size is a field;
 *   - get / has / set / delete build a key -> index hash table on their first
 *     use: open addressing in one Int32Array, FNV-1a over the key's character
 *     codes read straight from the packed string, candidates confirmed with
 *     startsWith at their offset -- no per-key string or Map entry is created;
 *   - the consumers' mutations (lib/kmerFinderClient.js:132-133 set 'db' /
 *     'collection', :223-225 and lib/kmerFinderServer.js:781-783 delete) follow
 *     Map semantics exactly: set on a present key keeps its position, a new (or
 *     deleted and re-set) key goes to the end, delete removes it.
 * Packed entries live in this object; keys added later live in the Map base
 * (super), which therefore holds exactly the entries appended after the
 * packed block, in insertion order.
 */
'use strict';

class KmerMap extends Map {
    // keys: a Latin-1 string of all keys back to back; off: n + 1 offsets;
    // cnt: n values (array-like); buf, indexer: the same keys as a Buffer and
    // the addon's indexKeys (builds _index's table natively), or absent
    constructor(keys, off, cnt, buf = null, indexer = null) {
        super();
        this._all = keys;
        this._buf = buf;
        this._indexer = indexer;
        this._off = off;
        this._cnt = cnt;
        this._n = cnt.length;
        this._tab = null;        // hash table of packed indices (built on first keyed access)
        this._mask = 0;
        this._mod = null;        // packed index -> value set since (Map)
        this._del = null;        // Uint8Array: packed index deleted
        this._ndel = 0;
    }

    static fromNative(res, indexer = null) {
        return new KmerMap('', [0], []).adopt(res, indexer);
    }

    // Become the packed native result `res` (replacing any content): how
    // readFile() fills the very Map object the constructor created, so that a
    // holder of this.kmerMap sees the counts (lib/kmers.js:76, :178 resolve the
    // constructor's Map).
    adopt(res, indexer = null) {
        super.clear();
        const n = res.counts.length;
        this._all = n ? res.keys.latin1Slice(0, res.offsets[n]) : '';
        this._buf = res.keys;
        this._indexer = indexer;
        this._off = res.offsets;
        this._cnt = res.counts;
        this._n = n;
        this._tab = null;
        this._mask = 0;
        this._mod = null;
        this._del = null;
        this._ndel = 0;
        return this;
    }

    _key(i) { return this._all.substring(this._off[i], this._off[i + 1]); }

    _value(i) {
        if (this._mod !== null) {
            const v = this._mod.get(i);
            if (v !== undefined || this._mod.has(i)) return v;
        }
        return this._cnt[i];
    }

    _live(i) { return this._del === null || this._del[i] === 0; }

    _hashAt(a, b) {
        const s = this._all;
        let h = 0x811c9dc5 | 0;
        for (let j = a; j < b; j += 1) h = Math.imul(h ^ s.charCodeAt(j), 16777619);
        return h;
    }

    _index() {
        if (this._tab === null) {
            const n = this._n;
            const off = this._off;
            let cap = 16;
            while (cap < 2 * n) cap *= 2;
            const mask = cap - 1;
            let tab;
            if (this._indexer !== null && this._buf !== null && off instanceof Float64Array) {
                tab = this._indexer(this._buf, off, n, cap);     // (the same table, built natively)
            } else {
                tab = new Int32Array(cap).fill(-1);
                for (let i = 0; i < n; i += 1) {
                    let h = this._hashAt(off[i], off[i + 1]) & mask;
                    while (tab[h] !== -1) h = (h + 1) & mask;
                    tab[h] = i;
                }
            }
            this._buf = null;            // (the string holds the keys from here on)
            this._tab = tab;
            this._mask = mask;
        }
        return this._tab;
    }

    // packed index of a live packed key, else -1
    _find(key) {
        if (typeof key !== 'string' || this._n === 0) return -1;
        const tab = this._index();
        const off = this._off;
        const all = this._all;
        let h = 0x811c9dc5 | 0;
        for (let j = 0; j < key.length; j += 1) h = Math.imul(h ^ key.charCodeAt(j), 16777619);
        h &= this._mask;
        for (let i = tab[h]; i !== -1; i = tab[h]) {
            if (off[i + 1] - off[i] === key.length && all.startsWith(key, off[i])) return this._live(i) ? i : -1;
            h = (h + 1) & this._mask;
        }
        return -1;
    }

    // the packed entries alone, unmodified (the matcher can take them as they are)
    _packedOnly() { return this._ndel === 0 && this._mod === null && super.size === 0; }

    // delete packed entry i (kmerfinder.js: the winners' k-mers, by index)
    _deletePacked(i) {
        if (!this._live(i)) return false;
        if (this._del === null) this._del = new Uint8Array(this._n);
        this._del[i] = 1;
        this._ndel += 1;
        if (this._mod !== null) this._mod.delete(i);
        return true;
    }

    get size() { return this._n - this._ndel + super.size; }

    get(key) {
        const i = this._find(key);
        return i >= 0 ? this._value(i) : super.get(key);
    }

    has(key) { return this._find(key) >= 0 || super.has(key); }

    set(key, value) {
        const i = this._find(key);
        if (i >= 0) {
            if (this._mod === null) this._mod = new Map();
            this._mod.set(i, value);
        } else {
            super.set(key, value);
        }
        return this;
    }

    delete(key) {
        const i = this._find(key);
        if (i < 0) return super.delete(key);
        if (this._del === null) this._del = new Uint8Array(this._n);
        this._del[i] = 1;
        this._ndel += 1;
        if (this._mod !== null) this._mod.delete(i);
        return true;
    }

    clear() {
        this._n = 0;
        this._buf = null;
        this._ndel = 0;
        this._all = '';
        this._tab = null;
        this._mod = null;
        this._del = null;
        super.clear();
    }

    * entries() {
        for (let i = 0; i < this._n; i += 1) if (this._live(i)) yield [this._key(i), this._value(i)];
        yield* super.entries();
    }

    * keys() {
        for (let i = 0; i < this._n; i += 1) if (this._live(i)) yield this._key(i);
        yield* super.keys();
    }

    * values() {
        for (let i = 0; i < this._n; i += 1) if (this._live(i)) yield this._value(i);
        yield* super.values();
    }

    [Symbol.iterator]() { return this.entries(); }

    forEach(fn, thisArg) {
        for (let i = 0; i < this._n; i += 1) if (this._live(i)) fn.call(thisArg, this._value(i), this._key(i), this);
        super.forEach((v, k) => fn.call(thisArg, v, k, this));
    }
}

module.exports = { KmerMap };
