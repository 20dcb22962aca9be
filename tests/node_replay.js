// Replays message logs through the Node host layer (fluidframework_amd/js) on the GPU and
// prints each document's text, property runs, SnapshotV1 blobs, status and digest as JSON.
// usage: node tests/node_replay.js <logs.json: [[msg, ...], ...]> [applyMsg|json]   (run by test_node_host.py)
// mode json: the native ingest (ReplayBatch.ingestJson -> mt_pack_json) instead of applyMsg
'use strict';
const fs = require('fs');
const path = require('path');
const { ReplayBatch } = require(path.join(__dirname, '..', 'fluidframework_amd', 'js'));

async function main() {
    const docs = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
    const batch = new ReplayBatch(docs.length);
    if (process.argv[3] === 'json') {
        batch.ingestJson(docs.map((msgs) => JSON.stringify(msgs)), 4);
    } else {
        docs.forEach((msgs, i) => {
            const c = batch.client(i);
            c.startOrUpdateCollaboration('readonly');
            for (const m of msgs) c.applyMsg(m);
        });
    }
    await batch.runAsync();
    const out = docs.map((_, i) => {
        const c = batch.client(i);
        if (c.status !== 0) return { status: c.status };
        return { status: 0, text: c.getText(), runs: c.propertyRuns(), snapshot: c.snapshotV1(),
                 digest: c.digest().toString(), props0: c.getPropertiesAtPosition(0) === undefined ? null : c.getPropertiesAtPosition(0) };
    });
    process.stdout.write(JSON.stringify(out));
}
main().catch((e) => { console.error(e); process.exit(1); });
