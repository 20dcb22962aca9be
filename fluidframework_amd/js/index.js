// index.js — Node host layer over libmtreplay.so (through the N-API addon mtreplay.node).
//
// Mirrors the reference's per-document merge-tree surface so a FluidFramework host can drop
// it in for the observer replay path:
//
//   reference (packages/dds/merge-tree/src, sequence/src)       here
//   -------------------------------------------------------      ---------------------------------------
//   new Client(specToSegment, logger)                            batch.client(i)  (a ReplayClient)
//   client.startOrUpdateCollaboration(longId)  (client.ts:1051)  client.startOrUpdateCollaboration(longId)
//   client.applyMsg(msg)                       (client.ts:797)   client.applyMsg(msg)   (queued), then
//                                                                batch.run() / await batch.runAsync()
//   client.getLength()                         (client.ts:1049)  client.getLength()
//   sharedString.getText()                     (sharedString.ts:211) client.getText()
//   client.getPropertiesAtPosition(pos)        (client.ts:1009)  client.getPropertiesAtPosition(pos)
//   new SnapshotV1(mt, logger).extractSync(); emit()             client.snapshotV1()  ({header, body_0..})
//   the Error applyMsg would throw                               client.status / client.error
//
// Every op is applied by the HIP kernel; this file only packs messages into the C ABI's
// records (include/mt_oplog.h).  Loading throws when the addon or the GPU is missing: there
// is no CPU fallback.
'use strict';

const path = require('path');

let addon = null;
function native() {
    if (!addon) addon = require(path.join(__dirname, 'mtreplay.node'));
    return addon;
}

const OP_INSERT = 0, OP_REMOVE = 1, OP_ANNOTATE = 2, OP_REGENERATE = 7, OP_NOOP = 15;
const OPF_GROUP_CONT = 1, OPF_MARKER = 2, OPF_HAS_PROPS = 4, OPF_REWRITE = 8;
const OP_RELPOS = 6, RELF_POS1 = 0x10, RELF_POS2 = 0x20, RELF_BEFORE1 = 0x40, RELF_BEFORE2 = 0x80, RELF_OFF1 = 0x100, RELF_OFF2 = 0x200;
const RELF_NOTIFY = 0x2;  // a local RELPOS of Client.annotateMarkerNotifyConsensus (include/mt_oplog.h)
const COMBINE_INCR = 1, COMBINE_CONSENSUS = 2, COMBINE_OTHER = 3, KEY_COMBINE = 0xFFFFFFFF, VALUE_UNDEFINED = 0xFFFFFFFF;
// an insert's prop count: flags bits 4-10 up to NPROPS_INLINE; beyond, NPROPS_EXT there and a first
// record {KEY_NPROPS, count} (include/mt_oplog.h MT_OPF_NPROPS_EXT)
const NPROPS_INLINE = 126, NPROPS_EXT = 127, KEY_NPROPS = 0xFFFFFFFE;
const MAX_CLIENTS = 0x7FFE;      // short ids 0..32765 (MT_MAX_CLIENTS; 0x7FFE / 0x7FFF are sentinels)
const STATUS = ['OK', 'INVALID_POS', 'SEQ_ORDER', 'MSN_ORDER', 'UNSUPPORTED', 'BAD_INPUT', 'CAPACITY', 'INTERNAL'];

class UnsupportedOp extends Error {}

// Packs ISequencedDocumentMessage streams (protocol.ts:132-172; ops.ts:29-110) into the
// 32-byte mt_op records, a UTF-16 text arena and interned property keys / values.  Short
// client ids follow Client.getOrAddShortClientId (client.ts:636-660): observer first, then
// first appearance.  Value ids intern JSON.stringify text; 0 is JSON null (delete).
class Packer {
    constructor(observer = 'readonly') {
        this.observer = observer;
        this.keys = [];
        this.values = ['null'];
        this.keyIds = new Map();
        this.valueIds = new Map([['null', 0]]);
        this.recs = [];
        this.textParts = [];
        this.textLen = 0;
        this.props = [];
        this.off = [0];
        this.clients = [];
    }
    key(k) {
        let i = this.keyIds.get(k);
        if (i === undefined) {
            i = this.keys.length;
            this.keyIds.set(k, i);
            this.keys.push(k);
        }
        return i;
    }
    value(v) {
        if (v === null || v === undefined) return 0;
        const s = JSON.stringify(v);
        let i = this.valueIds.get(s);
        if (i === undefined) {
            i = this.values.length;
            this.valueIds.set(s, i);
            this.values.push(s);
        }
        return i;
    }
    propRecords(props) {
        if (typeof props !== 'object' || props === null || Array.isArray(props)) throw new UnsupportedOp('props must be an object');
        const off = this.props.length / 2;
        for (const k of Object.keys(props)) this.props.push(this.key(k), this.value(props[k]));
        return [off, this.props.length / 2 - off];
    }
    // the marker id a Client.annotateMarkerNotifyConsensus op registers (client.ts:113-134): the op
    // createAnnotateMarkerOp makes (opBuilder.ts:25-39) with combiningOp {name: "consensus"}
    notifyId(members) {
        const op = members.length === 1 ? members[0] : null;
        const r1 = op && op.relativePos1, r2 = op && op.relativePos2, cop = op && op.combiningOp;
        const ok = op && op.type === OP_ANNOTATE && op.pos1 === undefined && op.pos2 === undefined &&
            cop && typeof cop === 'object' && Object.keys(cop).length === 1 && cop.name === 'consensus' &&
            r1 && r2 && typeof r1 === 'object' && typeof r2 === 'object' && r1.offset === undefined &&
            r2.offset === undefined && r1.id && typeof r1.id !== 'object' && r2.id === r1.id && r1.before && !r2.before;
        if (!ok) throw new UnsupportedOp('notifyConsensus on an op annotateMarkerNotifyConsensus does not make');
        return this.value(r1.id);
    }
    static flatten(op) {
        if (op.type === 3) return (op.ops || []).reduce((a, m) => a.concat(Packer.flatten(m)), []);
        return [op];
    }
    // the MT_OP_RELPOS record of an op whose pos1 (pos2) is undefined and relativePos1 (relativePos2)
    // truthy (Client.getValidOpRange, client.ts:485-502), else null
    relPos(op, base) {
        const r = Object.assign({}, base, { type: OP_RELPOS, flags: OPF_GROUP_CONT, pos1: 0, pos2: 0, payload: 0, payloadLen: 0 });
        for (const k of [1, 2]) {
            let rp = op[`relativePos${k}`];
            if (op[`pos${k}`] !== undefined || !rp || (k === 2 && op.type !== OP_REMOVE && op.type !== OP_ANNOTATE)) continue;
            r.flags |= k === 1 ? RELF_POS1 : RELF_POS2;
            if (typeof rp !== 'object' || Array.isArray(rp)) rp = {};
            if (rp.id) r[`pos${k}`] = this.value(rp.id);
            if (rp.before) r.flags |= k === 1 ? RELF_BEFORE1 : RELF_BEFORE2;
            if (Object.prototype.hasOwnProperty.call(rp, 'offset')) {  // `offset !== undefined`; null adds 0
                const off = rp.offset === null ? 0 : rp.offset;
                if (!Number.isInteger(off)) throw new UnsupportedOp('relative position offset must be an integer');
                r.flags |= k === 1 ? RELF_OFF1 : RELF_OFF2;
                r[k === 1 ? 'payload' : 'payloadLen'] = off >>> 0;
            }
        }
        return (r.flags & (RELF_POS1 | RELF_POS2)) ? r : null;
    }
    packOp(op, base) {
        const t = op.type;
        if (op.pos1 === undefined && !op.relativePos1) throw new UnsupportedOp('op without a position');
        if (op.register !== undefined) throw new UnsupportedOp('registers are not on the observer fast path');
        const r = Object.assign({}, base, { type: t, flags: 0, pos1: op.pos1 === undefined ? 0 : op.pos1 | 0, pos2: 0, payload: 0, payloadLen: 0 });
        if (t === OP_INSERT) {
            const seg = op.seg;
            let text = null, props;
            if (typeof seg === 'string') text = seg;
            else if (seg && typeof seg.text === 'string') { text = seg.text; props = seg.props; }
            else if (seg && seg.marker) {
                r.flags |= OPF_MARKER;
                r.payload = seg.marker.refType | 0;
                r.payloadLen = 1;
                props = seg.props;
            } else throw new UnsupportedOp('unknown segment spec');
            if (text !== null) {
                r.payload = this.textLen;
                r.payloadLen = text.length;  // UTF-16 code units, as TextSegment.cachedLength
                this.textParts.push(text);
                this.textLen += text.length;
            }
            if (Array.isArray(props)) throw new UnsupportedOp('array props');
            if (props && Object.keys(props).length) {  // TextSegment.make: `if (props) addProperties`
                let [off, n] = this.propRecords(props);
                if (n > NPROPS_INLINE) {  // any number of props: the count leads the records
                    this.props.splice(2 * off, 0, KEY_NPROPS, n);
                    n = NPROPS_EXT;
                }
                r.flags |= OPF_HAS_PROPS | (n << 4);
                r.pos2 = off;
            } else if (props && typeof props === 'object') {  // {} is truthy: an empty map
                r.flags |= OPF_HAS_PROPS;
                r.pos2 = this.props.length / 2;
            }
        } else if (t === OP_REMOVE || t === OP_ANNOTATE) {
            r.pos2 = (op.pos2 || 0) | 0;
            if (t === OP_ANNOTATE) {
                // addProperties (segmentPropertiesManager.ts:53-54): "rewrite", or Properties.combine
                // for any other truthy combiningOp (include/mt_oplog.h mt_combine_kind)
                const cop = op.combiningOp;
                let kind = 0;
                if (cop) {
                    if (cop.name === 'rewrite') r.flags |= OPF_REWRITE;
                    else kind = cop.name === 'incr' ? COMBINE_INCR : cop.name === 'consensus' ? COMBINE_CONSENSUS : COMBINE_OTHER;
                }
                // annotateRange -> addProperties(op.props) iterates its keys: an object is required
                [r.payload, r.payloadLen] = this.propRecords(op.props);
                if (kind) {
                    r.flags |= kind << 4;
                    const c = (typeof cop === 'object' && !Array.isArray(cop)) ? cop : {};
                    for (const f of ['defaultValue', 'minValue'])
                        this.props.push(KEY_COMBINE, Object.prototype.hasOwnProperty.call(c, f) ? this.value(c[f]) : VALUE_UNDEFINED);
                    this.props.push(KEY_COMBINE, VALUE_UNDEFINED);  // result slot (filled by the library)
                }
            }
        } else throw new UnsupportedOp(`op type ${t}`);
        return r;
    }
    addDocument(messages, observer = this.observer) {
        const names = [observer];
        const short = new Map([[observer, 0]]);
        const recs = [];
        for (let msg of messages) {
            if (typeof msg === 'string') msg = JSON.parse(msg);
            let c = short.get(msg.clientId);
            if (c === undefined) {
                if (names.length >= MAX_CLIENTS) throw new UnsupportedOp('more than 32765 clients (short ids are 15-bit)');
                c = names.length;
                short.set(msg.clientId, c);
                names.push(msg.clientId);
            }
            // a writer replica's own unsequenced message (sequenceNumber -1 = UnassignedSequenceNumber,
            // TestClient.makeOpMessage's default) is a local op; its sequenced ones ack them
            const local = msg.sequenceNumber === -1;
            const ack = c === 0 && !local;
            if (local && c !== 0) throw new UnsupportedOp('an unsequenced message of another client');
            const base = { client: c, seq: msg.sequenceNumber, refSeq: msg.referenceSequenceNumber || 0, msn: local ? 0 : msg.minimumSequenceNumber };
            const noop = Object.assign({}, base, { type: OP_NOOP, flags: 0, pos1: 0, pos2: 0, payload: 0, payloadLen: 0 });
            if (local && msg.type === 'regenerate') {
                // Client.regeneratePendingOp(contents, oldest pending group) on reconnect: one
                // MT_OP_REGENERATE record per member of the reset op (include/mt_oplog.h)
                const members = Packer.flatten(msg.contents);
                members.forEach((op, j) => {
                    const r = Object.assign({}, base, { type: OP_REGENERATE, refSeq: op.type, flags: 0, pos1: 0, pos2: 0, payload: 0, payloadLen: 0 });
                    if (op.type === OP_ANNOTATE) {
                        const cop = op.combiningOp;
                        if (cop) {
                            if (cop.name !== 'rewrite') throw new UnsupportedOp('local combiningOp other than rewrite');
                            r.flags |= OPF_REWRITE;
                        }
                        [r.payload, r.payloadLen] = this.propRecords(op.props);
                    } else if (op.type !== OP_INSERT && op.type !== OP_REMOVE) throw new UnsupportedOp(`regenerate of op type ${op.type}`);
                    if (j + 1 < members.length) r.flags |= OPF_GROUP_CONT;
                    recs.push(r);
                });
                continue;
            }
            if (msg.type !== 'op') {
                if (local) throw new UnsupportedOp('a local message that is not an op');
                recs.push(noop);
                continue;
            }
            const members = Packer.flatten(msg.contents);
            // {notifyConsensus: true} on a local message: the op came from
            // Client.annotateMarkerNotifyConsensus (a repo-defined field of the writer stream)
            const notify = local && !!msg.notifyConsensus;
            const notifyRaw = notify ? this.notifyId(members) : 0;
            members.forEach((op, j) => {
                const cop = op.combiningOp;
                const rel = this.relPos(op, base);
                if (rel && notify) {
                    rel.flags |= RELF_NOTIFY;
                    rel.payload = notifyRaw;
                }
                if (rel && !ack) recs.push(rel);  // an ack reads no positions
                // getValidOpRange validates an insert's end when one is given (client.ts:520-524)
                if (local && op.type === OP_INSERT && (op.pos2 !== undefined || op.relativePos2))
                    throw new UnsupportedOp('a local insert with an end position');
                const r = this.packOp(op, base);
                if (ack && op.type === OP_ANNOTATE && cop && cop.name === 'consensus') {
                    // updateConsensusProperty reads op.relativePos1.id (client.ts:981): a missing
                    // relativePos1 throws; an id a Map lookup cannot match (none, an object) is 0
                    const rp = op.relativePos1;
                    if (rp === undefined || rp === null) throw new UnsupportedOp('ack of a consensus annotate without relativePos1 (a TypeError)');
                    const id = rp.id;
                    r.pos1 = id === undefined || id === null || typeof id === 'object' ? 0 : this.value(id);
                }
                if (j + 1 < members.length) r.flags |= OPF_GROUP_CONT;
                recs.push(r);
            });
            if (!members.length) recs.push(noop);  // empty group: updateSeqNumbers only
        }
        for (const r of recs) this.recs.push(r);
        this.off.push(this.off[this.off.length - 1] + recs.length);
        this.clients.push(names);
    }
    finish() {
        const ops = Buffer.alloc(32 * Math.max(1, this.recs.length));
        this.recs.forEach((r, i) => {
            const o = 32 * i;
            // mt_op's type : 4, client : 12 (the id's low bits); its high 3 bits in flags 11-13
            ops.writeUInt16LE((r.type & 15) | ((r.client & 0xFFF) << 4), o);
            ops.writeUInt16LE(r.flags | (((r.client >> 12) & 7) << 11), o + 2);
            ops.writeInt32LE(r.seq, o + 4);
            ops.writeInt32LE(r.refSeq, o + 8);
            ops.writeInt32LE(r.msn, o + 12);
            ops.writeInt32LE(r.pos1, o + 16);
            ops.writeInt32LE(r.pos2, o + 20);
            ops.writeUInt32LE(r.payload >>> 0, o + 24);
            ops.writeUInt32LE(r.payloadLen >>> 0, o + 28);
        });
        const text = new Uint16Array(Math.max(1, this.textLen));
        let w = 0;
        for (const s of this.textParts) for (let i = 0; i < s.length; i++) text[w++] = s.charCodeAt(i);
        return {
            ops, docOpOff: BigInt64Array.from(this.off.map(BigInt)), text, nText: this.textLen,
            props: Uint32Array.from(this.props.length ? this.props : [0, 0]),
            keys: this.keys, values: this.values, clients: this.clients,
        };
    }
}

// One document of a batch: the merge-tree Client of an observer replica.
class ReplayClient {
    constructor(batch, index) {
        this.batch = batch;
        this.index = index;
        this.longClientId = 'readonly';
        this.messages = [];
    }
    startOrUpdateCollaboration(longClientId) { this.longClientId = longClientId; }
    applyMsg(msg) { this.batch.queued = true; this.messages.push(msg); }
    // A writer replica's local ops (Client.insertSegmentLocal / removeRangeLocal /
    // annotateRangeLocal, client.ts:201-291): queued as the replica's unsequenced messages
    // (sequenceNumber -1, as TestClient.makeOpMessage(op) builds them), applied on the GPU with
    // UnassignedSequenceNumber and acked when applyMsg later passes the replica's own sequenced
    // message.  Each returns the op, as the reference does.
    localOp(op) {
        this.batch.queued = true;
        this.messages.push({ clientId: this.longClientId, sequenceNumber: -1, referenceSequenceNumber: 0,
            minimumSequenceNumber: 0, type: 'op', contents: op });
        return op;
    }
    insertTextLocal(pos, text, props) { return this.localOp({ pos1: pos, seg: props ? { text, props } : text, type: OP_INSERT }); }
    insertMarkerLocal(pos, refType, props) {
        return this.localOp({ pos1: pos, seg: props ? { marker: { refType }, props } : { marker: { refType } }, type: OP_INSERT });
    }
    removeRangeLocal(start, end) { return this.localOp({ pos1: start, pos2: end, type: OP_REMOVE }); }
    annotateRangeLocal(start, end, props, combiningOp) {
        const op = { pos1: start, pos2: end, props, type: OP_ANNOTATE };
        if (combiningOp) op.combiningOp = combiningOp;
        return this.localOp(op);
    }
    // Client.annotateMarkerNotifyConsensus(marker, props, callback) (client.ts:113-134), the marker
    // named by its id: createAnnotateMarkerOp's op queued as a local message marked
    // notifyConsensus.  The replay records each callback the reference would make (the ack's
    // updateConsensusProperty, then minSeq reaching its seq); runConsensusCallbacks() makes them,
    // in order, after run(), with the marker id and the seq / minSeq of the call.
    annotateMarkerNotifyConsensus(markerId, props, callback) {
        const op = { combiningOp: { name: 'consensus' }, props, relativePos1: { id: markerId, before: true },
            relativePos2: { id: markerId }, type: OP_ANNOTATE };
        this.batch.queued = true;
        this.messages.push({ clientId: this.longClientId, sequenceNumber: -1, referenceSequenceNumber: 0,
            minimumSequenceNumber: 0, type: 'op', contents: op, notifyConsensus: true });
        if (callback) {
            if (!this.consensusCallbacks) this.consensusCallbacks = new Map();
            this.consensusCallbacks.set(markerId, callback);  // pendingConsensus.set (client.ts:129)
        }
        return op;
    }
    consensusEvents() { return JSON.parse(native().docConsensusEvents(this.batch.h, this.index)); }
    runConsensusCallbacks() {
        for (const e of this.consensusEvents()) {
            const cb = this.consensusCallbacks && this.consensusCallbacks.get(e.markerId);
            if (cb) cb(e);
        }
    }
    // Client.regeneratePendingOp(resetOp, ...) on reconnect (client.ts:855-893): queued; the
    // regenerated ops come back from regeneratedOps() after run()
    regeneratePendingOp(resetOp) {
        this.batch.queued = true;
        this.messages.push({ clientId: this.longClientId, sequenceNumber: -1, type: 'regenerate', contents: resetOp });
    }
    regeneratedOps() { return JSON.parse(native().docRegeneratedOps(this.batch.h, this.index)); }
    // Client.findTile(startPos, tileLabel, preceding = true) (client.ts:1073-1076) on the final state
    findTile(startPos, tileLabel, preceding = true) {
        const r = native().docFindTile(this.batch.h, this.index, startPos, tileLabel, preceding);
        return r === undefined ? undefined : { pos: r.pos, props: r.props ? JSON.parse(r.props) : undefined };
    }
    // Client.getStackContext(startPos, rangeLabels) (client.ts:946-948; SharedSegmentSequence
    // .getStackContext, sequence.ts:377): { label: [{ pos, refType, props }] }, stacks bottom to top
    getStackContext(startPos, rangeLabels) {
        return JSON.parse(native().docStackContext(this.batch.h, this.index, startPos, rangeLabels));
    }
    get status() { return native().docStatus(this.batch.h, this.index); }
    get error() { const s = this.status; return s === 0 ? undefined : STATUS[s] || String(s); }
    getText() { return native().docText(this.batch.h, this.index); }
    getLength() { return this.getText().length; }
    // [start, length, JSON.stringify(props) | null] per run of equal properties over the text
    propertyRuns() { return JSON.parse(native().docPropsRuns(this.batch.h, this.index)); }
    getPropertiesAtPosition(pos) {
        for (const [start, len, props] of this.propertyRuns())
            if (start <= pos && pos < start + len) return props === null ? undefined : JSON.parse(props);
        return undefined;
    }
    snapshotV1() { return native().docSnapshotV1(this.batch.h, this.index); }
    digest() { return native().docDigest(this.batch.h, this.index); }
}

// A batch of SharedString documents replayed on the current MI355X.
class ReplayBatch {
    constructor(nDocs, options = {}) {
        this.nDocs = nDocs;
        this.h = native().createBatch(nDocs, options);
        this.clients = Array.from({ length: nDocs }, (_, i) => new ReplayClient(this, i));
        this.queued = false;
    }
    client(i) { return this.clients[i]; }
    // messages queued through client(i).applyMsg -> one packed upload
    flush() {
        if (!this.queued) return;
        const p = new Packer();
        for (const c of this.clients) p.addDocument(c.messages, c.longClientId);
        this.ingestPacked(p.finish());
        this.queued = false;
    }
    ingestPacked(pb) {
        const n = native();
        n.setTables(this.h, pb.keys.length ? pb.keys : ['_'], pb.values);
        const shared = pb.clients.every((c) => JSON.stringify(c) === JSON.stringify(pb.clients[0]));
        if (shared && pb.clients.length) n.setClients(this.h, -1, pb.clients[0]);
        else pb.clients.forEach((c, i) => n.setClients(this.h, i, c));
        n.ingest(this.h, pb.ops, pb.docOpOff, pb.text.subarray(0, Math.max(1, pb.nText)), pb.props);
    }
    // native ingest: per document the JSON text of its message array (the file driver's
    // messages.json) or the array itself; device 'auto' parses on the GPU (mt_json_gpu.hip) and
    // falls back to the host parser (mt_pack_json) outside its fast path, 'gpu' / 'host' force one.
    // Returns the parser that ran ('gpu' | 'host').
    ingestJson(docs, nThreads = 0, device = 'auto') {
        if (docs.length !== this.nDocs) {  // the native parsers read exactly nDocs documents
            const e = new RangeError(`ingestJson: ${docs.length} documents for a batch of ${this.nDocs}`);
            e.code = 101;  // MT_ERR_ARG
            throw e;
        }
        const texts = docs.map((d) => (typeof d === 'string' ? d : JSON.stringify(d)));
        const path = native().ingestJson(this.h, texts, this.clients.length ? this.clients[0].longClientId : 'readonly',
                                         nThreads, device);
        this.queued = false;
        for (const c of this.clients) c.messages = [];
        return path;
    }
    ingestMessages(docs) {
        docs.forEach((msgs, i) => { for (const m of msgs) this.clients[i].applyMsg(m); });
        this.flush();
    }
    generate(params, docFirst = 0) { native().generate(this.h, params, docFirst); }
    run() { this.flush(); native().run(this.h); }
    runAsync() { this.flush(); return native().runAsync(this.h); }
    stats() { return native().stats(this.h); }
    deviceDigests() {
        const out = new BigUint64Array(this.nDocs);
        native().deviceDigests(this.h, out);
        return out;
    }
}

module.exports = { ReplayBatch, ReplayClient, Packer, UnsupportedOp, STATUS, native };
