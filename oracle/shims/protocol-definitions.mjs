// TEST INFRASTRUCTURE ONLY: enums from server/routerlicious/packages/protocol-definitions
// (protocol.ts:6-60 MessageType, storage.ts:28-34 FileMode, storage.ts:73-77 TreeEntry).
export const MessageType = {
    NoOp: "noop", ClientJoin: "join", ClientLeave: "leave", Propose: "propose", Reject: "reject",
    Summarize: "summarize", SummaryAck: "summaryAck", SummaryNack: "summaryNack", Operation: "op",
    Save: "saveOp", Fork: "fork", Integrate: "integrate", RemoteHelp: "remoteHelp",
};
export const FileMode = { File: "100644", Executable: "100755", Directory: "040000",
    Commit: "160000", Symlink: "120000" };
export const TreeEntry = { Blob: "Blob", Commit: "Commit", Tree: "Tree" };
