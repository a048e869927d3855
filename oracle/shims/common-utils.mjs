// TEST INFRASTRUCTURE ONLY: minimal stand-in for @fluidframework/common-utils as used by
// the transpiled reference merge-tree (Trace: common/lib/common-utils/src/trace.ts:12-33;
// base64: common/lib/common-utils/src/base64Encoding.ts:8).
import { performance } from "perf_hooks";
export class Trace {
    static start() { return new Trace(performance.now()); }
    constructor(startTick) { this.startTick = startTick; this.lastTick = startTick; }
    trace() {
        const tick = performance.now();
        const ev = { totalTimeElapsed: tick - this.startTick, duration: tick - this.lastTick, tick };
        this.lastTick = tick;
        return ev;
    }
}
export const fromBase64ToUtf8 = (s) => Buffer.from(s, "base64").toString("utf8");
export const fromUtf8ToBase64 = (s) => Buffer.from(s, "utf8").toString("base64");
export const IsoBuffer = Buffer;
