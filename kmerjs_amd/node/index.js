/* index.js — drop-in for kmerjs's npm main (package.json:14 -> dist/index.js,
 * built from lib/index.js), backed by the MI355X counter.
 *
 * Same exports as lib/index.js: kmers, complement (the legacy line loop and
 * reverse complement, :60-73, :97-101), KmerJSClient and KmerJSServer
 * (:324-354, :398-467) over the legacy KmerJS base (:216-248: fields fastq,
 * preffix, length, step, out, coverage, uKmers, db {type, url}, evalue;
 * stringToMap / objectToMap / mapToJSON, the latter returning a JSON string).
 *
 * findKmers() is the reference's readLinesBrowser (:250-306): '\n' lines, the
 * line counter mod 4, `i === 1 && line.length > 1` selects a sequence line,
 * kmers() over the line and over complement(line).  Here the whole file is
 * counted by the GPU (kmer_count_file) and the promise resolves to the same
 * Map<kmer, count>, in the same first-occurrence order (a KmerMap, filled
 * lazily).  Divergences, error and diagnostic paths only: the per-line
 * progress line and the 'ERROR!' / 'ERROR2!' header checks (console output
 * only in the reference) are not printed; a File (browser) input of
 * KmerJSClient is not served (the GPU addon reads paths); findMatches --
 * template matching against the kmerFinder MongoDB / HTTP service -- is out of
 * this build's scope and rejects.
 */
'use strict';
const path = require('path');
const drop = require('./kmers.js');

const { KmerMap, complement, kmers } = drop;

const dbs = new Map([
    ['mongo', 'mongodb://localhost:27017/Kmers'],
    ['json', '../test_data/db.json'],
]);

function objToStrMap(obj) {
    const m = new Map();
    for (const k of Object.keys(obj)) m.set(k, obj[k]);
    return m;
}

// readLinesBrowser(kmerObj, reader) on the GPU: resolves to the Map
function countPath(kmerObj, fastq) {
    return new Promise((resolve, reject) => {
        if (typeof fastq !== 'string') {
            reject(new Error('kmerjs_amd: findKmers needs a file path (browser File input is not served)'));
            return;
        }
        let handle;
        try {
            handle = drop.native().open(kmerObj.length, Buffer.from(String(kmerObj.preffix), 'latin1'),
                kmerObj.step, Number(process.env.KMERHIP_DEVICE || 0), 0, kmerObj.maxKeys, 0, drop.devices(kmerObj));
        } catch (e) {
            reject(e);
            return;
        }
        drop.native().countFile(handle, path.resolve(fastq), (err, res) => {
            drop.native().close(handle);
            if (err) {
                if (err.status === 5) {
                    const e = new RangeError(err.message);
                    e.status = 5;
                    reject(e);
                } else {
                    reject(err);
                }
                return;
            }
            let map;
            try {
                map = KmerMap.fromNative(res, drop.native().indexKeys);
            } catch (e) {
                reject(e);
                return;
            }
            // (readLinesBrowser, lib/index.js:250-306, sets neither uKmers nor
            // a line count on the object: only the unused readLineNode does, :389)
            resolve(map);
        });
    });
}

class KmerJS {
    constructor(fastq, preffix = 'ATGAC', length = 16, step = 1, coverage = 1, out = '', db = 'mongo') {
        this.fastq = fastq;
        this.preffix = preffix;
        this.length = length;
        this.step = step;
        this.out = out === '' ? undefined : out;
        this.coverage = coverage;
        this.uKmers = 0;
        this.db = { type: db, url: dbs.get(db) };
        this.evalue = new drop.KmerJS().evalue;     // BN(0.05), with .cmp()
        this.maxKeys = 16777216;                    // the Map's limit (lib/index.js:70, Map.set)
    }

    stringToMap(string) { return objToStrMap(JSON.parse(string)); }

    objectToMap(object) { return objToStrMap(object); }

    mapToJSON(strMap) {
        const obj = Object.create(null);
        for (const [k, v] of strMap) obj[k] = v;
        return JSON.stringify(obj);
    }
}

class KmerJSClient extends KmerJS {
    constructor(fastq, preffix = 'ATGAC', length = 16, step = 1, coverage = 1, out = '', db = 'mongo',
        url = 'http://localhost:3000/kmers') {
        super(fastq, preffix, length, step, coverage, out, db);
        this.url = url;
    }

    findKmers() { return countPath(this, this.fastq); }

    findMatches() {
        return Promise.reject(new Error('kmerjs_amd: findMatches (kmerFinder template service) is out of scope'));
    }
}

class KmerJSServer extends KmerJS {
    findKmers() { return countPath(this, this.fastq); }

    findMatches() {
        return Promise.reject(new Error('kmerjs_amd: findMatches (kmerFinder MongoDB templates) is out of scope'));
    }
}

module.exports = { kmers, complement, KmerJSClient, KmerJSServer };
