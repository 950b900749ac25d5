// End-to-end readFile() -> Map through the Node drop-in (SURVEY.md §8d (iii)):
// file on disk -> kmer_count_file (host read, H2D, GPU count, ordered result
// D2H) -> N-API -> KmerMap; then the consumer-side costs: a full iteration
// (lib/kmerFinderServer.js:175), the first keyed access (index build,
// :798-799), and for comparison an eager copy into a plain Map.
// usage: node tools/e2e_readfile.js FILE [prefix] [k]
'use strict';
const path = require('path');
const { KmerJS } = require(path.join(__dirname, '..', 'kmerjs_amd', 'node', 'kmers.js'));

(async () => {
    const file = process.argv[2];
    const prefix = process.argv[3] === undefined ? 'ATGAC' : process.argv[3];
    const k = Number(process.argv[4] || 16);
    const now = () => Number(process.hrtime.bigint()) / 1e6;
    // warm-up: device init, addon load
    await new KmerJS(path.join(__dirname, '..', 'tests', 'golden', 'inputs', 'test_short.fastq'), prefix, k, 1, 1, false).readFile().promise;
    const t0 = now();
    const kj = new KmerJS(file, prefix, k, 1, 1, false);
    const map = await kj.readFile().promise;
    const t1 = now();
    let sum = 0, first = null;
    for (const [key, v] of map) { if (first === null) first = key; sum += v; }
    const t2 = now();
    const hit = map.get(first);
    const t3 = now();
    const eager = new Map(map);
    const t4 = now();
    process.stdout.write(JSON.stringify({
        readfile_ms: t1 - t0, iterate_ms: t2 - t1, first_get_ms: t3 - t2, eager_map_ms: t4 - t3,
        size: map.size, sum, lines: kj.lines, first_count: hit, eager_size: eager.size,
        per_entry_us: { readfile: (t1 - t0) * 1e3 / map.size, iterate: (t2 - t1) * 1e3 / map.size,
            index: (t3 - t2) * 1e3 / map.size, eager: (t4 - t3) * 1e3 / map.size },
    }) + '\n');
})().catch((e) => { console.error(e); process.exit(1); });
