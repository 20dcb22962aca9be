// index.d.ts — TypeScript declarations of the Node host layer (index.js) over libmtreplay.so.
// Method names follow the reference Client (packages/dds/merge-tree/src/client.ts).

/** ISequencedDocumentMessage fields the observer replay reads (protocol.ts:132-172). */
export interface ISequencedDocumentMessage {
    clientId: string;
    sequenceNumber: number;
    referenceSequenceNumber: number;
    minimumSequenceNumber: number;
    type: string;
    contents: any;  // IMergeTreeOp (ops.ts:29-110) when type === "op"
}

export interface BatchOptions { segCap?: number; maxRetries?: number; }

export interface GenParams {
    nOps: number; nClients?: number; maxLag?: number; pctInsert?: number; pctRemove?: number;
    minLen?: number; maxInsert?: number; pctNewline?: number; seed?: number;
}

export declare const STATUS: string[];
export declare class UnsupportedOp extends Error {}

export declare class ReplayClient {
    readonly index: number;
    /** Client.startOrUpdateCollaboration(longClientId) (client.ts:1051): the observer's id. */
    startOrUpdateCollaboration(longClientId: string): void;
    /** Client.applyMsg(msg) (client.ts:797): queued; applied on the GPU by ReplayBatch.run().
     *  The replica's own sequenced messages ack its pending local ops. */
    applyMsg(msg: ISequencedDocumentMessage | string): void;
    /** Writer replicas: Client.insertSegmentLocal / removeRangeLocal / annotateRangeLocal
     *  (client.ts:201-291), queued as unsequenced messages (sequenceNumber -1); returns the op. */
    insertTextLocal(pos: number, text: string, props?: Record<string, any>): object;
    insertMarkerLocal(pos: number, refType: number, props?: Record<string, any>): object;
    removeRangeLocal(start: number, end: number): object;
    annotateRangeLocal(start: number, end: number, props: Record<string, any>, combiningOp?: { name: string }): object;
    /** Client.annotateMarkerNotifyConsensus(marker, props, callback) (client.ts:113-134) on the marker
     *  with this id; the callback runs from runConsensusCallbacks() after run(). */
    annotateMarkerNotifyConsensus(markerId: string, props: Record<string, any>,
                                  callback?: (e: { markerId: any; seq: number; minSeq: number }) => void): object;
    /** the consensus callbacks the replay made, in call order (after run()). */
    consensusEvents(): { markerId: any; seq: number; minSeq: number }[];
    runConsensusCallbacks(): void;
    /** Client.regeneratePendingOp(resetOp, oldest pending group) on reconnect (client.ts:855-893). */
    regeneratePendingOp(resetOp: object): void;
    /** the regenerated ops of every regeneratePendingOp call, in order (after run()). */
    regeneratedOps(): object[];
    /** Client.findTile(startPos, tileLabel, preceding) (client.ts:1073-1076) on the final state. */
    findTile(startPos: number, tileLabel: string, preceding?: boolean): { pos: number; props?: Record<string, any> } | undefined;
    /** Client.getStackContext(startPos, rangeLabels) (client.ts:946-948) on the final state: range
     *  label -> its NestBegin / NestEnd markers, bottom to top. */
    getStackContext(startPos: number, rangeLabels: string[]): Record<string, { pos: number; refType: number; props?: Record<string, any> }[]>;
    /** 0 = OK, else the MT_* status of the Error applyMsg would have thrown. */
    readonly status: number;
    readonly error: string | undefined;
    getText(): string;
    getLength(): number;
    getPropertiesAtPosition(pos: number): Record<string, any> | undefined;
    propertyRuns(): Array<[number, number, string | null]>;
    /** new SnapshotV1(mergeTree, logger).extractSync(); emit(): blob name -> utf-8 JSON. */
    snapshotV1(): Record<string, string>;
    digest(): bigint;
}

export declare class ReplayBatch {
    constructor(nDocs: number, options?: BatchOptions);
    readonly nDocs: number;
    client(i: number): ReplayClient;
    ingestMessages(docs: Array<Array<ISequencedDocumentMessage | string>>): void;
    /** Native parse + pack (mt_pack_json on nThreads host threads, 0 = all cores) of each
     *  document's message array, given as its JSON text (messages.json) or as the array. */
    ingestJson(docs: Array<string | ISequencedDocumentMessage[]>, nThreads?: number,
               device?: 'auto' | 'gpu' | 'host'): 'gpu' | 'host';
    generate(params: GenParams, docFirst?: number): void;
    run(): void;
    runAsync(): Promise<void>;
    stats(): { nDocs: number; nOps: number; opsApplied: number; docsFailed: number; launches: number;
               kernelMs: number; totalMs: number; ldsBytes: number };
    deviceDigests(): BigUint64Array;
}
