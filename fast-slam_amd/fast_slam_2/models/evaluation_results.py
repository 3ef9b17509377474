"""Evaluation result record (reference: fast_slam_2/models/evaluation_results.py), the
`results` block of the serializer's JSON."""


class EvaluationResults:
    def __init__(self, timestamp: str, average_deviation: float, x_deviation: float, y_deviation: float,
                 angular_deviation: float, distance: float):
        self.timestamp = timestamp
        self.average_deviation = average_deviation
        self.x_deviation = x_deviation
        self.y_deviation = y_deviation
        self.angular_deviation = angular_deviation
        self.distance = distance

    def to_dict(self) -> dict:
        return {
            "timestamp": self.timestamp,
            "average_deviation": self.average_deviation,
            "x_deviation": self.x_deviation,
            "y_deviation": self.y_deviation,
            "angular_deviation": self.angular_deviation,
            "distance": self.distance,
        }
