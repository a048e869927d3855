// TEST INFRASTRUCTURE ONLY: no-op loggers standing in for @fluidframework/telemetry-utils.
const noop = {
    send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {},
    logGenericError() {}, logException() {}, debugAssert() {}, shipAssert() {},
};
export class ChildLogger { static create() { return noop; } }
export class DebugLogger { static create() { return noop; } }
